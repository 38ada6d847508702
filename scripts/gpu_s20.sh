# The driver's shape, fresh process each: --steps 20 --warmup 5 (N runs per
# variant), with the host enqueue / HIP-event split of each line.
# usage: bash scripts/gpu_s20.sh TAG [N]
TAG=${1:-s20}; N=${2:-5}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for i in $(seq $N); do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $OUT/s20_default.jsonl 2>&1 || exit $?
done
for i in $(seq $N); do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --warmup-spl 5 --no-cpu-baseline >> $OUT/s20_warm1launch.jsonl 2>&1 || exit $?
done
