# Round 6: direct server commands (the default) -- server tests, the
# driver-shape bench A/B against the relay form (PBH_SERVER_DIRECT=0,
# interleaved), the per-command device stamps of both, then the GPU suite,
# smoke and both bench shapes.  usage: bash scripts/gpu_r06q.sh TAG
export TMPDIR=/tmp
TAG=${1:-r06q}
OUT=gpurun_out/$TAG
mkdir -p $OUT
sha256sum probayes_amd/libpbhip.so > $OUT/lib.sha256
T="python -u -m pytest -q -rf -p no:warnings --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_server.py > $OUT/tests_server.log 2>&1 || exit $?
for i in 1 2 3 4; do
for d in 1 0; do
timeout -k 10 200 env PBH_SERVER_DIRECT=$d python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-replay --no-launched > $OUT/s20_direct${d}_$i.jsonl 2>&1 || exit $?
done
done
timeout -k 10 120 env PBH_SERVER_DIRECT=1 python scripts/server_probe.py 65536 20 > $OUT/probe_direct1.jsonl 2>&1 || exit $?
timeout -k 10 120 env PBH_SERVER_DIRECT=0 python scripts/server_probe.py 65536 20 > $OUT/probe_direct0.jsonl 2>&1 || exit $?
timeout -k 10 600 $T tests -m gpu > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_workloads.py --no-cpu-baseline --only cfg5 > $OUT/cfg5.jsonl 2>&1 || exit $?
timeout -k 10 300 python bench.py > $OUT/bench_default.jsonl 2> $OUT/bench_default.err || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.jsonl 2> $OUT/bench_driver.err || exit $?
