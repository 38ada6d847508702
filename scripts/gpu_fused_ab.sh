#!/bin/bash
# Fused REPLAY A/B of a variant library against the shipped one: the legacy
# and fused parity suites on the variant, then interleaved fused / two-kernel
# probes and generator timings, then one SQ pass each.
# usage: bash scripts/gpu_fused_ab.sh <tag> <variant .so under probayes_amd/>
T=${1:-fab}; V=${2:-libpbhip_ab.so}
mkdir -p gpurun_out/$T
PBHIP_LIB=$PWD/probayes_amd/$V timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_legacy.py tests/test_gpu_legacy_fused.py > gpurun_out/$T/tests.log 2>&1 || exit $?
for rep in 1 2; do
  for lib in libpbhip.so $V; do
    PBHIP_LIB=$PWD/probayes_amd/$lib timeout -k 10 100 python -u scripts/replay_fused_probe.py 65536 1000 250 fused | sed "s/^/$lib /" >> gpurun_out/$T/probe.txt || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp
for lib in libpbhip.so $V; do
  PBHIP_LIB=$OLDPWD/probayes_amd/$lib timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY --output-format csv -d $OLDPWD/gpurun_out/$T/sq_$lib -o run -- python3 $OLDPWD/scripts/replay_fused_probe.py 65536 500 250 > $OLDPWD/gpurun_out/$T/sq_$lib.log 2>&1 || exit $?
done
