# The headline bench in fresh processes: the driver's shape 5 times, the
# default shape 3 times (no CPU baseline)
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/rep_s20.jsonl gpurun_out/rep_def.jsonl
for i in 1 2 3 4 5; do timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> gpurun_out/rep_s20.jsonl 2>&1 || exit $?; done
for i in 1 2 3; do timeout -k 10 120 python bench.py --no-cpu-baseline >> gpurun_out/rep_def.jsonl 2>&1 || exit $?; done
