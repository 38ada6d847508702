# legacy streams: tests, wall-time probe, and a kernel trace of the probe
export TMPDIR=/tmp
R=$PWD
mkdir -p gpurun_out/legtr
timeout -k 10 300 python -u -m pytest tests/test_gpu_legacy.py -m gpu -x -q -p no:warnings --timeout 120 --timeout-method thread > gpurun_out/leg_tests.log 2>&1 || exit $?
timeout -k 10 200 python scripts/probe_legacy.py > gpurun_out/leg_probe.jsonl 2>&1 || exit $?
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/legtr -o run -- python3 $R/scripts/probe_legacy.py > $R/gpurun_out/legtr/probe.log 2>&1
