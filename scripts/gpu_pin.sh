# driver-shape bench with the rank pinned to its CPU (PBH_BENCH_PIN=1) or not,
# interleaved
export TMPDIR=/tmp
OUT=gpurun_out/pin
mkdir -p $OUT
for i in 1 2 3 4 5 6; do
for p in 1 0; do
timeout -k 10 120 env PBH_BENCH_PIN=$p python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-replay --no-launched >> $OUT/pin$p.jsonl 2>/dev/null || exit $?
done
done
