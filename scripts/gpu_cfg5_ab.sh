# cfg5 quad kernel: parity tests, then the workload line 3 times
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pd.py -m gpu -x -q -p no:warnings --timeout 120 --timeout-method thread -k "gmm or quad or pd" > gpurun_out/c5_tests.log 2>&1 || exit $?
for i in 1 2 3; do timeout -k 10 120 python scripts/bench_workloads.py --no-cpu-baseline --only cfg5 >> gpurun_out/c5_wl.jsonl 2>&1 || exit $?; done
