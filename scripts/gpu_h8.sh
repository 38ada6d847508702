# the fused REPLAY kernel's window at H = 8 (libpbhip.so) against H = 16
# (libpbhip_base.so), interleaved; then the fused tests on the H = 8 build
export TMPDIR=/tmp
OUT=gpurun_out/h8
mkdir -p $OUT
for i in 1 2 3; do
timeout -k 10 120 python scripts/replay_fused_probe.py 65536 1000 250 fused >> $OUT/h8.jsonl 2>&1 || exit $?
timeout -k 10 120 env PBHIP_LIB=$PWD/probayes_amd/libpbhip_base.so python scripts/replay_fused_probe.py 65536 1000 250 fused >> $OUT/h16.jsonl 2>&1 || exit $?
done
timeout -k 10 300 python -u -m pytest -x -q -p no:warnings --timeout 120 --timeout-method thread tests/test_gpu_legacy_fused.py > $OUT/tests.log 2>&1 || exit $?
