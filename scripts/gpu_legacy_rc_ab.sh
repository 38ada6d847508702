#!/bin/bash
# Window-refill A/B (PBH_LEGACY_RC): the shipped library (one-chunk refills)
# against probayes_amd/libpbhip_ab.so (built with -DPBH_LEGACY_RC=2, the
# round-4 two-chunk refills), interleaved: the fused / two-kernel probe and
# the generator alone; then the legacy and fused parity suites on the shipped
# library.  usage: bash scripts/gpu_legacy_rc_ab.sh <tag>
T=${1:-rcab}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_legacy.py tests/test_gpu_legacy_fused.py > gpurun_out/$T/tests.log 2>&1 || exit $?
for rep in 1 2; do
  for lib in libpbhip.so libpbhip_ab.so; do
    PBHIP_LIB=$PWD/probayes_amd/$lib timeout -k 10 100 python -u scripts/replay_fused_probe.py 65536 1000 250 fused,two_kernel | sed "s/^/$lib /" >> gpurun_out/$T/probe.txt || exit $?
    PBHIP_LIB=$PWD/probayes_amd/$lib timeout -k 10 100 python -u scripts/legacy_kernel.py 65536 250 4 | sed "s/^/$lib /" >> gpurun_out/$T/gen.txt || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp
for lib in libpbhip.so libpbhip_ab.so; do
  PBHIP_LIB=$OLDPWD/probayes_amd/$lib timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY --output-format csv -d $OLDPWD/gpurun_out/$T/sq_$lib -o run -- python3 $OLDPWD/scripts/replay_fused_probe.py 65536 500 250 > $OLDPWD/gpurun_out/$T/sq_$lib.log 2>&1 || exit $?
done
