# Effective clock (GRBM_GUI_ACTIVE / 8 XCDs / kernel time) and SQ activity of
# the cfg2 kernel, with and without the trace, per RNG mode.
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/pmc_clock_$1
rm -rf $OUT && mkdir -p $OUT
cd /tmp
for RNG in $2; do
  for TR in "" "--no-trace"; do
    N=${RNG}${TR}
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/$N -o run -- python3 $R/bench.py --steps 500 --warmup 250 --no-cpu-baseline --rng $RNG $TR > $OUT/$N.log 2>&1 || exit 1
  done
done
