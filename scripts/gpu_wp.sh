# The word-parallel legacy generator: parity suites, then timings against the
# chain-per-lane generator (PBH_LEGACY_WP=0) and the fused kernel.
export TMPDIR=/tmp
TAG=${1:-r06b}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_legacy_wp.py tests/test_gpu_legacy.py tests/test_gpu_legacy_fused.py tests/test_sp_api.py tests/test_facade.py -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 120 env PBH_LEGACY_WP=1 python scripts/legacy_kernel.py > $OUT/gen_wp.jsonl 2>&1 || exit $?
timeout -k 10 120 env PBH_LEGACY_WP=0 python scripts/legacy_kernel.py > $OUT/gen_mt4.jsonl 2>&1 || exit $?
timeout -k 10 200 env PBH_LEGACY_WP=1 python scripts/replay_fused_probe.py 65536 1000 250 fused,two_kernel > $OUT/replay_forms.jsonl 2>&1 || exit $?
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace -o run -- python3 $GRAFT_REPO_ROOT/scripts/replay_fused_probe.py 65536 1000 250 two_kernel > $GRAFT_REPO_ROOT/$OUT/trace.log 2>&1 || exit $?
