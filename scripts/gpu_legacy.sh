export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_legacy.py tests/test_facade.py tests/test_gpu_parity.py -m gpu -q -rf -p no:warnings --timeout 120 --timeout-method thread -k "legacy or batched or full_width or device_streams" > gpurun_out/${1}_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${1}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python scripts/probe_legacy.py > gpurun_out/${1}_legacy.jsonl 2>&1 || exit $?
exit $rc
