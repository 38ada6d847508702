# PMC passes over the device legacy-stream generator (gauss)
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/pmc_leg
rm -rf $OUT && mkdir -p $OUT
cd /tmp
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d $OUT/p$i -o run -- python3 $R/scripts/probe_legacy_one.py gauss > $OUT/p$i.log 2>&1 || exit $?
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/scripts/probe_legacy_one.py gauss > $OUT/trace.log 2>&1 || exit $?
python3 $R/scripts/pmc_summary.py $OUT legacy 250 > $R/gpurun_out/pmc_leg_summary.txt 2>&1
