# GPU tests + bench lines (philox, xoshiro); logs under gpurun_out/.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rf -p no:warnings --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/gpu_tests.log
timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --no-cpu-baseline --rng xoshiro >> gpurun_out/bench.log 2>&1 || exit 1
