# twist-ahead for the chain-per-lane stream generator: legacy tests, then
# gibbs8 stream generation with the pass on / off, interleaved
export TMPDIR=/tmp
OUT=gpurun_out/gen_ahead
mkdir -p $OUT
sha256sum probayes_amd/libpbhip.so > $OUT/lib.sha256
timeout -k 10 400 python -u -m pytest -x -q -p no:warnings --timeout 120 --timeout-method thread tests/test_gpu_legacy.py tests/test_gpu_legacy_fused.py tests/test_gpu_legacy_wp.py tests/test_linreg.py tests/test_facade.py > $OUT/tests.log 2>&1 || exit $?
for i in 1 2; do
for a in 1 0; do
timeout -k 10 120 env PBH_LEGACY_AHEAD=$a python scripts/legacy_gen_probe.py 32768 256 4 >> $OUT/gen_ahead$a.jsonl 2>&1 || exit $?
done
done
