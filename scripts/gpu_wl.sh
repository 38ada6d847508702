# GPU tests of the MH kernels, then the secondary workloads (cfg1/cfg3/cfg5)
export TMPDIR=/tmp
TAG=${1:-wl}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -rf -p no:warnings --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python scripts/bench_workloads.py --only cfg5,cfg1,cfg3 --no-cpu-baseline > gpurun_out/${TAG}_wl.jsonl 2>&1 || exit 1
PBH_GMM_LANES=2 timeout -k 10 300 python scripts/bench_workloads.py --only cfg5 --no-cpu-baseline >> gpurun_out/${TAG}_wl.jsonl 2>&1 || exit 1
exit $rc
