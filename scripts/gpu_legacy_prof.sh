# legacy streams: tests, wall-time probe, and a kernel trace of the probe
export TMPDIR=/tmp
R=$PWD
bash scripts/gpu_legacy_win.sh || exit $?
mkdir -p gpurun_out/legtr
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/legtr -o run -- python3 $R/scripts/probe_legacy.py > $R/gpurun_out/legtr/probe.log 2>&1
