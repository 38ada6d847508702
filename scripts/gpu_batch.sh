# One GPU session: tests, driver-shape bench, workloads, cfg5 PMC passes.
export TMPDIR=/tmp
TAG=${1:-batch}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -rf -p no:warnings --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
timeout -k 10 120 python bench.py --no-cpu-baseline >> gpurun_out/${TAG}_bench.log 2>&1 || exit $?
timeout -k 10 120 python bench.py --no-cpu-baseline --rng philox_fp32 >> gpurun_out/${TAG}_bench.log 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_workloads.py --only cfg5,cfg1,cfg3 --no-cpu-baseline > gpurun_out/${TAG}_wl.jsonl 2>&1 || exit $?
bash scripts/pmc_cmd.sh ${TAG}_gmmq scripts/bench_workloads.py --only cfg5 --no-cpu-baseline || exit $?
exit $rc
