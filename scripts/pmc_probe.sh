# PMC passes (one rocprofv3 run per counter group) of bench.py's cfg2 kernel
# for each RNG mode given: issue / stall / LDS split.
# usage: bash scripts/pmc_probe.sh TAG "philox philox_fp32"
export TMPDIR=/tmp
R=$PWD
TAG=$1
OUT=$R/gpurun_out/pmc_$TAG
rm -rf $OUT && mkdir -p $OUT
cd /tmp
for RNG in $2; do
  ARGS="--steps 500 --warmup 250 --no-cpu-baseline --rng $RNG"
  i=0
  for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_LDS" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/${RNG}_p$i -o run -- python3 $R/bench.py $ARGS > $OUT/${RNG}_p$i.log 2>&1 || exit 1
  done
done
python3 $R/scripts/pmc_summary.py $OUT mh_pair > $OUT/summary.txt
