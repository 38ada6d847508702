# cfg2 headline: parity tests of the MH kernels, then the bench at the
# default and the driver's shapes (twice each)
export TMPDIR=/tmp
TAG=${1:-c2}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_accept_filter.py -m gpu -x -q -p no:warnings --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit $?
for i in 1 2; do
timeout -k 10 120 python bench.py --no-cpu-baseline >> gpurun_out/${TAG}_bench.jsonl 2>&1 || exit $?
timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 5 >> gpurun_out/${TAG}_bench_s20.jsonl 2>&1 || exit $?
done
