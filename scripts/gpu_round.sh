# One GPU call: GPU parity tests, smoke, bench (philox and xoshiro).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rf -p no:warnings --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 180 python bench.py > gpurun_out/bench.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --rng xoshiro --no-cpu-baseline >> gpurun_out/bench.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --no-cpu-baseline --chains 131072 >> gpurun_out/bench.log 2>&1
