export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_normals.py -m gpu -q -rf -p no:warnings --timeout 120 --timeout-method thread > gpurun_out/${1}_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${1}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/${1}_bench.jsonl 2>&1 || exit $?
exit $rc
