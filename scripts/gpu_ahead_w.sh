# twist-ahead workgroup width A/B (PBH_AHEAD_W = 4 / 8 / 16), interleaved,
# plus the kernel trace at each width
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/ahead_w
mkdir -p $OUT
R=$PWD
timeout -k 10 300 python -u -m pytest -x -q -p no:warnings --timeout 120 --timeout-method thread tests/test_gpu_legacy_fused.py > $OUT/tests.log 2>&1 || exit $?
for i in 1 2; do
for w in 4 8 16; do
timeout -k 10 120 env PBH_AHEAD_W=$w python scripts/replay_fused_probe.py 65536 1000 250 fused >> $OUT/w$w.jsonl 2>&1 || exit $?
done
done
cd /tmp
for w in 4 16; do
timeout -k 10 200 env PBH_AHEAD_W=$w rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace$w -o run -- python3 $R/scripts/replay_fused_probe.py 65536 1000 250 fused > $OUT/trace$w.log 2>&1 || exit $?
done
