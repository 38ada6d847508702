# cfg5 quad kernel: FULL vs general timing, kernel trace, SQ PMC pass
export TMPDIR=/tmp
R=$PWD; T=${1:-c5}
mkdir -p gpurun_out/$T
for f in 1 0 1 0; do
  PBH_GMM_FULL=$f timeout -k 10 60 python3 scripts/cfg5_kernel.py >> gpurun_out/${T}/full$f.txt 2>&1 || exit $?
done
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$T/trace -o run -- python3 $R/scripts/cfg5_kernel.py > $R/gpurun_out/$T/trace.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY --output-format csv -d $R/gpurun_out/$T/sq -o run -- python3 $R/scripts/cfg5_kernel.py > $R/gpurun_out/$T/sq.log 2>&1
