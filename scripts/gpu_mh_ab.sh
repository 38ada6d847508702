# mh_kernel paths: GPU tests, then the cfg1 workload lines
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/mh_wl.jsonl
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:warnings --timeout 120 --timeout-method thread > gpurun_out/mh_tests.log 2>&1 || exit $?
for i in 1 2; do timeout -k 10 120 python scripts/bench_workloads.py --no-cpu-baseline --only cfg1,cfg5 >> gpurun_out/mh_wl.jsonl 2>&1 || exit $?; done
