# PMC passes for the lane-pair bench kernel: issue vs stall split.
set -e
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/pmc
rm -rf $OUT && mkdir -p $OUT
ARGS="--steps 500 --warmup 250 --no-cpu-baseline"
cd /tmp
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_WR GRBM_GUI_ACTIVE"; do
  N=$(echo $C | tr ' ' '_' | cut -c1-40)
  timeout -k 10 200 rocprofv3 --pmc $C --output-format csv -d $OUT/$N -o run -- python3 $R/bench.py $ARGS > $OUT/$N.log 2>&1
done
