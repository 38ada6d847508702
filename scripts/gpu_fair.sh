#!/bin/bash
# A/B of the wave-priority alternation (PBH_FAIR) on the FULL pair kernel:
# phase stamps (probe build) and bench lines at both launch shapes.
# usage: bash scripts/gpu_fair.sh TAG
set -o pipefail
T=${1:-fair}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for F in 1 0; do
  PBH_FAIR=$F PBHIP_LIB=probayes_amd/libpbhip_ph.so PHASE_RAW=gpurun_out/${T}_f${F}_phase_raw.npz \
    timeout -k 10 240 python3 -u scripts/phase_probe.py "${T}_f$F" > gpurun_out/${T}_f${F}_phase.jsonl 2> gpurun_out/${T}_f${F}_phase.err || exit $?
done
for F in 1 0; do
  PHASE_WORKLOAD=gmm2 PBH_FAIR=$F PBHIP_LIB=probayes_amd/libpbhip_ph.so PHASE_RAW=gpurun_out/${T}_g${F}_phase_raw.npz \
    timeout -k 10 240 python3 -u scripts/phase_probe.py "${T}_g$F" > gpurun_out/${T}_g${F}_phase.jsonl 2> gpurun_out/${T}_g${F}_phase.err || exit $?
done
for i in 1 2; do for F in 1 0; do
  PBH_FAIR=$F timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> gpurun_out/${T}_f${F}_s20.jsonl 2>> gpurun_out/${T}_bench.err || exit $?
  PBH_FAIR=$F timeout -k 10 120 python3 bench.py --gpus 1 --steps 1000 --warmup 250 >> gpurun_out/${T}_f${F}_s1000.jsonl 2>> gpurun_out/${T}_bench.err || exit $?
done; done
