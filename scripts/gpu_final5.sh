# Round-5 evidence at HEAD: GPU suite, smoke, workload lines, the headline's
# rocprofv3 passes (scripts/profile_r05.sh -> gpurun_out/prof5) and cfg5's
# kernel trace + SQ pass.  usage: bash scripts/gpu_final5.sh TAG
export TMPDIR=/tmp
TAG=${1:-fin5}
mkdir -p gpurun_out/$TAG
timeout -k 10 500 python -u -m pytest tests -m gpu -q -rf -p no:warnings --timeout 120 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$TAG/smoke.log 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_workloads.py --no-cpu-baseline > gpurun_out/$TAG/workloads.jsonl 2>&1 || exit $?
bash scripts/profile_r05.sh || exit $?
bash scripts/gpu_cfg5.sh $TAG/c5
