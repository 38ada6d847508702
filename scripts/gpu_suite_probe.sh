# Full GPU test suite, the cfg5 workload, then the legacy-stream probe.
export TMPDIR=/tmp
TAG=${1:-s}
bash scripts/gpu_quick2.sh $TAG
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python scripts/probe_legacy.py > gpurun_out/${TAG}_legacy.jsonl 2>&1 || exit $?
exit $rc
