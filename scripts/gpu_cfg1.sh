# cfg1 steady-state kernel at 65 536 chains: lane-pair vs one-lane timing,
# kernel trace and an SQ PMC pass of each
export TMPDIR=/tmp
R=$PWD; T=${1:-c1}
mkdir -p gpurun_out/$T
for f in 1 0 1 0; do
  PBH_IID_PAIR=$f timeout -k 10 60 python3 scripts/cfg1_kernel.py >> gpurun_out/${T}/pair$f.txt 2>&1 || exit $?
done
cd /tmp
for f in 1 0; do
  PBH_IID_PAIR=$f timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY --output-format csv -d $R/gpurun_out/$T/sq$f -o run -- python3 $R/scripts/cfg1_kernel.py > $R/gpurun_out/$T/sq$f.log 2>&1 || exit $?
done
