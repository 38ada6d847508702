# cfg5 iteration: the GMM kernels' tests, the workload line, PMC passes
TAG=${1:-cfg5}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "gmm" -q -p no:warnings --timeout 120 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 || { tail -20 gpurun_out/$TAG/tests.log; exit 1; }
tail -1 gpurun_out/$TAG/tests.log
for i in 1 2; do timeout -k 10 300 python scripts/bench_workloads.py --no-cpu-baseline --only cfg5 >> gpurun_out/$TAG/wl.jsonl 2>&1 || exit $?; done
bash scripts/gpu_pmc_kernel.sh $TAG python3 /root/repo/scripts/cfg5_kernel.py
