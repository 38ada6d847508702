# Round-2 GPU iteration: tests (no -x: see every failure), launch probe, the
# driver's bench shape.  Stops at any crash / timeout (rc other than 0 or 1).
export TMPDIR=/tmp
TAG=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -rf -p no:warnings --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/launch_probe.py > gpurun_out/${TAG}_probe.jsonl 2> gpurun_out/${TAG}_probe.err || exit $?
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
timeout -k 10 120 python bench.py --no-cpu-baseline >> gpurun_out/${TAG}_bench.log 2>&1 || exit $?
exit $rc
