export TMPDIR=/tmp
OUT=gpurun_out/summary
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q -rf -p no:warnings --timeout 120 --timeout-method thread tests/test_facade.py tests/test_sp_api.py tests/test_gpu_pd.py tests/test_linreg.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 300 python scripts/facade_workload.py 65536 1000 2 250 walk > $OUT/facade_workload.jsonl 2>&1 || exit $?
