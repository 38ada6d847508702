# A/B of the kernel-form switches on the current build (workload lines)
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/var_*.jsonl
timeout -k 10 120 python scripts/bench_workloads.py --no-cpu-baseline --only cfg3,cfg5,linreg > gpurun_out/var_def.jsonl 2>&1 || exit $?
PBH_GIBBS_LANES=4 timeout -k 10 120 python scripts/bench_workloads.py --no-cpu-baseline --only cfg3 > gpurun_out/var_gl4.jsonl 2>&1 || exit $?
PBH_GIBBS_LANES=1 timeout -k 10 120 python scripts/bench_workloads.py --no-cpu-baseline --only cfg3 > gpurun_out/var_gl1.jsonl 2>&1 || exit $?
PBH_GMM_LANES=2 timeout -k 10 120 python scripts/bench_workloads.py --no-cpu-baseline --only cfg5 > gpurun_out/var_gm2.jsonl 2>&1 || exit $?
PBH_LINREG_PAIR=1 timeout -k 10 120 python scripts/bench_workloads.py --no-cpu-baseline --only linreg > gpurun_out/var_lrp.jsonl 2>&1 || exit $?
timeout -k 10 120 python scripts/bench_workloads.py --no-cpu-baseline --only cfg3,cfg5,linreg > gpurun_out/var_def2.jsonl 2>&1 || exit $?
