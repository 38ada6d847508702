# Headline kernel evidence on one box: the bench at the driver's shape
# (--steps 20 --warmup 5, fresh process each) and the default shape, then
# SQ PMC passes of mh_pair_kernel (issue, stalls, LDS) at 500 steps.
# usage: bash scripts/gpu_headline.sh TAG [extra bench args]
export TMPDIR=/tmp
TAG=${1:-hl}; shift
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT && rm -rf $OUT/pmc $OUT/s20.jsonl $OUT/s1000.jsonl
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" >> $OUT/s20.jsonl 2>&1 || exit $?
done
for i in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu-baseline "$@" >> $OUT/s1000.jsonl 2>&1 || exit $?
done
cd /tmp
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_LDS" \
         "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc/p$i -o run -- python3 $R/bench.py --steps 500 --warmup 250 --no-cpu-baseline "$@" > $OUT/pmc_p$i.log 2>&1 || exit $?
done
cd $R
python3 scripts/pmc_summary.py $OUT/pmc mh_pair_kernel 250 > $OUT/pmc_summary.txt 2>&1
