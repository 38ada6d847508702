# linreg Gibbs: tests, then the workload line 3 times
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_linreg.py -m gpu -x -q -p no:warnings --timeout 120 --timeout-method thread > gpurun_out/lr_tests.log 2>&1 || exit $?
for i in 1 2 3; do timeout -k 10 120 python scripts/bench_workloads.py --no-cpu-baseline --only linreg >> gpurun_out/lr_wl.jsonl 2>&1 || exit $?; done
