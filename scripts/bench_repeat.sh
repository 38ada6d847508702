# The headline bench at the driver's shape, repeated (fresh process each).
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3 4 5; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> gpurun_out/${1}_s20.jsonl 2>&1 || exit $?
done
for i in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu-baseline >> gpurun_out/${1}_s1000.jsonl 2>&1 || exit $?
done
