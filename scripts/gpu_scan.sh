export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -q -rf -p no:warnings > gpurun_out/gpu_tests.log 2>&1; echo "pytest rc=$?" >> gpurun_out/gpu_tests.log
rm -f gpurun_out/bench_scan.log
for n in 65536 131072 262144; do timeout -k 10 120 python bench.py --steps 500 --warmup 20 --no-cpu-baseline --chains $n >> gpurun_out/bench_scan.log 2>&1 || break; done
timeout -k 10 120 python bench.py --steps 500 --warmup 20 --no-cpu-baseline --no-trace >> gpurun_out/bench_scan.log 2>&1
timeout -k 10 120 python bench.py --steps 500 --warmup 20 --no-cpu-baseline --rng philox_f64 >> gpurun_out/bench_scan.log 2>&1
