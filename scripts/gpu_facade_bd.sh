export TMPDIR=/tmp
mkdir -p gpurun_out/facade_bd
for m in walk iter walk iter; do
timeout -k 10 200 python scripts/facade_workload.py 65536 1000 3 250 $m >> gpurun_out/facade_bd/facade_workload_$m.jsonl 2>&1 || exit $?
done
timeout -k 10 200 python bench.py --steps 1000 --warmup 250 --no-cpu-baseline --no-launched > gpurun_out/facade_bd/bench_replay.jsonl 2>&1 || exit $?
