# PMC passes (one rocprofv3 run per counter group) of any python command.
# usage: bash scripts/pmc_cmd.sh TAG script.py [args...]   (script relative to the repo)
export TMPDIR=/tmp
R=$PWD
TAG=$1; SCRIPT=$R/$2; shift 2
OUT=$R/gpurun_out/pmc_$TAG
rm -rf $OUT && mkdir -p $OUT
cd /tmp
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
         "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $OUT/run_p$i -o run -- python3 $SCRIPT "$@" > $OUT/p$i.log 2>&1 || exit 1
done
