# s20_probe.py in fresh processes, plain and under a few variants.
TAG=${1:-s20p}
OUT=gpurun_out/$TAG
mkdir -p $OUT
run() { t=$1; shift; env "$@" timeout -k 10 120 python scripts/s20_probe.py $t >> $OUT/s20probe.jsonl 2>>$OUT/s20probe.err || exit $?; }
for i in 1 2 3; do
  run base
  run prime PROBE_PRIME=1
  run warm16 PROBE_WARM=16
  run pin PROBE_PIN=1
  run nogc PROBE_GC=0
  run kernarg0 HIP_FORCE_DEV_KERNARG=0
done
