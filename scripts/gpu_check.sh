# One GPU call: tests, smoke, bench lines, workload bench, rocprof + PMC.
# Each GPU step has its own time limit; a crash/abort/timeout ends the call.
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out
mkdir -p $O
step() {  # step <name> <seconds> <cmd...>
  local n=$1 t=$2; shift 2
  echo "== $n: $*" >> $O/steps.log
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "== $n rc=$rc" >> $O/steps.log
  case $rc in 124|134|137|139) echo "fatal rc=$rc in $n"; exit $rc;; esac
  return 0
}
step tests 420 python -u -m pytest tests -m gpu -x -q -rf -p no:warnings --timeout 120 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
step bench 240 python bench.py
step bench_xo 120 python bench.py --rng xoshiro --no-cpu-baseline
step workloads 240 python scripts/bench_workloads.py
[ -x tools/ubench/isa_cost ] && step isa_cost 120 tools/ubench/isa_cost
[ -x tools/ubench/store_pattern ] && step store_pattern 120 tools/ubench/store_pattern
step gibbs_lanes4 120 env PBH_GIBBS_LANES=4 python scripts/bench_workloads.py --only cfg3 --no-cpu-baseline
step gibbs_ndtri 120 env PBH_GIBBS_FAST=0 python scripts/bench_workloads.py --only cfg3 --no-cpu-baseline
step gibbs_ndtri_valu 120 env PBH_GIBBS_FAST=0 PBH_GIBBS_MFMA=0 python scripts/bench_workloads.py --only cfg3 --no-cpu-baseline
step gmm_lanes4 120 env PBH_GMM_LANES=4 python scripts/bench_workloads.py --only cfg5 --no-cpu-baseline
P=$O/prof; mkdir -p $P; cd /tmp
A="--steps 1000 --warmup 250 --no-cpu-baseline"
step prof_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python3 $R/bench.py $A
step prof_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -o run -- python3 $R/bench.py $A
step prof_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/write -o run -- python3 $R/bench.py $A
step prof_sq1 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR --output-format csv -d $P/sq1 -o run -- python3 $R/bench.py $A
step prof_sq2 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --output-format csv -d $P/sq2 -o run -- python3 $R/bench.py $A
step prof_sq3 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_WR GRBM_GUI_ACTIVE --output-format csv -d $P/sq3 -o run -- python3 $R/bench.py $A
step prof_wl 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/wl -o run -- python3 $R/scripts/bench_workloads.py --no-cpu-baseline
step prof_wl_fetch 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/wl_fetch -o run -- python3 $R/scripts/bench_workloads.py --only cfg3 --no-cpu-baseline
step prof_wl_write 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/wl_write -o run -- python3 $R/scripts/bench_workloads.py --only cfg3 --no-cpu-baseline
step prof_lik_fetch 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/lik_fetch -o run -- python3 $R/scripts/bench_workloads.py --only lik --no-cpu-baseline
step prof_lik_write 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/lik_write -o run -- python3 $R/scripts/bench_workloads.py --only lik --no-cpu-baseline
echo done
