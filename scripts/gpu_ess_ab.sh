# device ESS of the cfg5 trace: wall per PBH_ESS_FFT mode (2: one-wave
# 2 048-point form, 3: two-wave 2 048-point form, 1: 4 096-point form), then a
# kernel trace and SQ passes of the default
export TMPDIR=/tmp
R=$PWD; T=${1:-ess}
mkdir -p gpurun_out/$T
for m in 2 3 1 2 3 1; do
  echo "mode $m" >> gpurun_out/$T/wall.txt
  PBH_ESS_FFT=$m timeout -k 10 120 python3 scripts/ess_kernel.py >> gpurun_out/$T/wall.txt 2>&1 || exit $?
done
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$T/trace -o run -- python3 $R/scripts/ess_kernel.py > $R/gpurun_out/$T/trace.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY --output-format csv -d $R/gpurun_out/$T/sq -o run -- python3 $R/scripts/ess_kernel.py > $R/gpurun_out/$T/sq.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_INSTS_VMEM_RD --output-format csv -d $R/gpurun_out/$T/sq2 -o run -- python3 $R/scripts/ess_kernel.py > $R/gpurun_out/$T/sq2.log 2>&1
