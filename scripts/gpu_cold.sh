# the in-kernel twist round out of line (mt4_twist_cold): legacy tests, the
# fused probe with twist-ahead on (x3) and off (x1)
export TMPDIR=/tmp
OUT=gpurun_out/cold
mkdir -p $OUT
sha256sum probayes_amd/libpbhip.so > $OUT/lib.sha256
timeout -k 10 400 python -u -m pytest -x -q -p no:warnings --timeout 120 --timeout-method thread tests/test_gpu_legacy.py tests/test_gpu_legacy_fused.py tests/test_gpu_legacy_wp.py tests/test_linreg.py > $OUT/tests.log 2>&1 || exit $?
for i in 1 2 3; do
timeout -k 10 120 python scripts/replay_fused_probe.py 65536 1000 250 fused >> $OUT/ahead1.jsonl 2>&1 || exit $?
done
timeout -k 10 120 env PBH_LEGACY_AHEAD=0 python scripts/replay_fused_probe.py 65536 1000 250 fused >> $OUT/ahead0.jsonl 2>&1 || exit $?
timeout -k 10 120 env PBH_LEGACY_FUSED=0 python scripts/replay_fused_probe.py 65536 1000 250 two_kernel >> $OUT/two_kernel.jsonl 2>&1 || exit $?
