# Round-6 evidence at HEAD: GPU suite, smoke, workload lines, the seeded
# facade workload, the fused REPLAY probe (twist-ahead on / off), then the
# headline's rocprofv3 passes (scripts/profile_r06.sh -> gpurun_out/prof6).
# usage: bash scripts/gpu_final6.sh TAG
export TMPDIR=/tmp
TAG=${1:-fin6}
OUT=gpurun_out/$TAG
mkdir -p $OUT
sha256sum probayes_amd/libpbhip.so > $OUT/lib.sha256
T="python -u -m pytest -q -rf -p no:warnings --timeout 120 --timeout-method thread"
timeout -k 10 500 $T tests -m gpu > $OUT/tests.log 2>&1 || exit $?
tail -1 $OUT/tests.log > $OUT/tests_summary.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_workloads.py --no-cpu-baseline > $OUT/workloads.jsonl 2>&1 || exit $?
timeout -k 10 200 python scripts/facade_workload.py 65536 1000 3 250 > $OUT/facade_workload.jsonl 2>&1 || exit $?
for a in 1 0; do
timeout -k 10 120 env PBH_LEGACY_AHEAD=$a python scripts/replay_fused_probe.py 65536 1000 250 fused >> $OUT/replay_ahead$a.jsonl 2>&1 || exit $?
done
bash scripts/profile_r06.sh || exit $?
