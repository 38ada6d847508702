# device ESS (FFT kernel) of the cfg5 trace: wall, kernel trace, SQ passes
export TMPDIR=/tmp
R=$PWD; T=${1:-ess}
mkdir -p gpurun_out/$T
timeout -k 10 120 python3 scripts/ess_kernel.py > gpurun_out/$T/wall.txt 2>&1 || exit $?
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$T/trace -o run -- python3 $R/scripts/ess_kernel.py > $R/gpurun_out/$T/trace.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY --output-format csv -d $R/gpurun_out/$T/sq -o run -- python3 $R/scripts/ess_kernel.py > $R/gpurun_out/$T/sq.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_INSTS_VMEM_RD --output-format csv -d $R/gpurun_out/$T/sq2 -o run -- python3 $R/scripts/ess_kernel.py > $R/gpurun_out/$T/sq2.log 2>&1
