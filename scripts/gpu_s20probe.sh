# s20_probe.py in fresh processes (the first timed launch after the warm-up),
# the lane-pair kernels' GPU tests, and the bench at the driver's shape
TAG=${1:-s20p}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_normals.py -q -x -k "pair or normals or diag10 or bench" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2 3 4; do
  PROBE_WARMLOOP=1 timeout -k 10 120 python scripts/s20_probe.py warmloop >> $OUT/s20probe.jsonl 2>>$OUT/s20probe.err || exit $?
done
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $OUT/s20_bench.jsonl 2>&1 || exit $?
done
