# Round 6: Mt4 with 16 buffers + the twist-ahead pass before fused REPLAY
# launches -- the legacy-stream tests, then the fused REPLAY probe with the
# pass on and off (PBH_LEGACY_AHEAD), interleaved
export TMPDIR=/tmp
OUT=gpurun_out/ahead
mkdir -p $OUT
sha256sum probayes_amd/libpbhip.so > $OUT/lib.sha256
T="python -u -m pytest -x -q -rf -p no:warnings --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_legacy.py tests/test_gpu_legacy_fused.py tests/test_gpu_legacy_wp.py tests/test_facade.py > $OUT/tests.log 2>&1 || exit $?
for i in 1 2; do
for a in 1 0; do
timeout -k 10 120 env PBH_LEGACY_AHEAD=$a python scripts/replay_fused_probe.py 65536 1000 250 fused >> $OUT/ahead$a.jsonl 2>&1 || exit $?
done
done
R=$PWD
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/trace -o run -- python3 $R/scripts/replay_fused_probe.py 65536 1000 250 fused > $R/$OUT/trace.log 2>&1 || exit $?
