# production Gibbs: tests, then the cfg3 workload twice
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/gb_wl.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_gibbs_fast.py tests/test_gpu_parity.py tests/test_facade.py -m gpu -x -q -p no:warnings --timeout 120 --timeout-method thread > gpurun_out/gb_tests.log 2>&1 || exit $?
for i in 1 2; do timeout -k 10 120 python scripts/bench_workloads.py --no-cpu-baseline --only cfg3 >> gpurun_out/gb_wl.jsonl 2>&1 || exit $?; done
