# s20_probe.py in fresh processes: the first timed launch after the warm-up
TAG=${1:-s20p}
OUT=gpurun_out/$TAG
mkdir -p $OUT
run() { t=$1; shift; env "$@" timeout -k 10 120 python scripts/s20_probe.py $t >> $OUT/s20probe.jsonl 2>>$OUT/s20probe.err || exit $?; }
for i in 1 2 3 4; do
  run warmloop PROBE_WARMLOOP=1
  run modlaunch PROBE_WARMLOOP=1 PBH_MODULE_LAUNCH=1
done
PBH_MODULE_LAUNCH=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "pair_steady or iid_steady or gmm_quad_steady" --timeout 120 --timeout-method thread > $OUT/modlaunch_tests.log 2>&1 || exit $?
