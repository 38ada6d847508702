# timing-only: the fused REPLAY kernel with the MT19937 generator replaced
# by a counter hash (PBH_LEGACY_FAKE=1) against the real one
export TMPDIR=/tmp
OUT=gpurun_out/fake
mkdir -p $OUT
for i in 1 2; do
timeout -k 10 120 env PBH_LEGACY_FAKE=1 python scripts/replay_fused_probe.py 65536 1000 250 fused >> $OUT/fake.jsonl 2>&1 || exit $?
timeout -k 10 120 env PBH_LEGACY_FAKE=0 python scripts/replay_fused_probe.py 65536 1000 250 fused >> $OUT/real.jsonl 2>&1 || exit $?
done
