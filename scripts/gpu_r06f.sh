# thresholds in the fused kernel, the façade's seeded path through it, the
# device linreg draws: the suites that cover them, then the workload line
export TMPDIR=/tmp
TAG=${1:-r06f}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_facade.py tests/test_sp_api.py tests/test_linreg.py tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/facade_workload.py 65536 1000 3 > $OUT/facade.jsonl 2>&1 || exit $?
timeout -k 10 200 env PBH_LEGACY_WP=1 python scripts/replay_fused_probe.py 65536 1000 250 fused > $OUT/replay.jsonl 2>&1 || exit $?
