# Full GPU suite, then every workload line (no CPU baselines) and the
# headline bench at the driver's and the default shapes.
export TMPDIR=/tmp
TAG=${1:-f}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -rf -p no:warnings --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python scripts/bench_workloads.py --no-cpu-baseline > gpurun_out/${TAG}_wl.jsonl 2>&1 || exit $?
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench_s20.jsonl 2>&1 || exit $?
timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.jsonl 2>&1 || exit $?
exit $rc
