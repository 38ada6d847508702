export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_legacy.py tests/test_gpu_parity.py tests/test_facade.py -m gpu -x -q -p no:warnings --timeout 120 --timeout-method thread > gpurun_out/leg_tests.log 2>&1 || exit $?
timeout -k 10 200 python scripts/probe_legacy.py > gpurun_out/leg_probe.jsonl 2>&1 || exit $?
PBH_LEGACY_WIN=0 timeout -k 10 200 python scripts/probe_legacy.py > gpurun_out/leg_probe_nowin.jsonl 2>&1
