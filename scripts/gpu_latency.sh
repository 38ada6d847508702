# Short-launch latency A/B: launch_probe.py's wall / enqueue / event time of
# 1- and 20-step launches (cfg2, 65 536 chains) in a fresh process per
# variant (runtime knobs are read at HIP / engine init).
# usage: bash scripts/gpu_latency.sh TAG
TAG=${1:-lat}
OUT=gpurun_out/$TAG
mkdir -p $OUT
run() { tag=$1; shift; env "$@" timeout -k 10 120 python scripts/launch_probe.py $tag 1,20 >> $OUT/latency.jsonl 2>>$OUT/latency.err || exit $?; }
run base
run full0 PBH_PAIR_FULL=0
run nofence PBH_EVENT_FLAGS=0x20000000
run devkernarg1 HIP_FORCE_DEV_KERNARG=1
run devkernarg0 HIP_FORCE_DEV_KERNARG=0
run nomarkers PBH_EVENT_MARKERS=0
run base2
