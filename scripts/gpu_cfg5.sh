# cfg5 quad kernel: parity tests touching the GMM kernels, then the cfg5
# workload line with the steady-state form on and off.
export TMPDIR=/tmp
TAG=${1:-c5}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q -rf -p no:warnings --timeout 120 --timeout-method thread -k "gmm or expectation or quantile or trace" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python scripts/bench_workloads.py --only cfg5 --no-cpu-baseline > gpurun_out/${TAG}_wl_full.jsonl 2>&1 || exit $?
PBH_GMM_FULL=0 timeout -k 10 200 python scripts/bench_workloads.py --only cfg5 --no-cpu-baseline > gpurun_out/${TAG}_wl_general.jsonl 2>&1 || exit $?
exit $rc
