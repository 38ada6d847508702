# s20_probe.py in fresh processes: the first timed launch after the warm-up
TAG=${1:-s20p}
OUT=gpurun_out/$TAG
mkdir -p $OUT
run() { t=$1; shift; env "$@" timeout -k 10 120 python scripts/s20_probe.py $t >> $OUT/s20probe.jsonl 2>>$OUT/s20probe.err || exit $?; }
for i in 1 2 3 4; do
  run warmloop PROBE_WARMLOOP=1
  run syncevent PROBE_WARMLOOP=1 PBH_SYNC=event
  run reldevice PROBE_WARMLOOP=1 PBH_EVENT_FLAGS=0x40000000
done
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $OUT/s20_bench.jsonl 2>&1 || exit $?
done
