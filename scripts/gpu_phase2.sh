#!/bin/bash
# Quarter-progress phase stamps: cfg2 / gmm2 at full width (two waves per SIMD)
# and at half width (one), with and without PBH_FAIR.  usage: gpu_phase2.sh TAG
set -o pipefail
T=${1:-ph}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {   # name, env...
  local name=$1; shift
  env "$@" PBHIP_LIB=probayes_amd/libpbhip_ph.so PHASE_RAW=gpurun_out/${T}_${name}_raw.npz \
    timeout -k 10 240 python3 -u scripts/phase_probe.py "${T}_$name" > gpurun_out/${T}_${name}.jsonl 2> gpurun_out/${T}_${name}.err
}
run c2f1 PBH_FAIR=1 && run c2f0 PBH_FAIR=0 && run c2h PBH_FAIR=0 PHASE_N=32768 && \
run g2f1 PBH_FAIR=1 PHASE_WORKLOAD=gmm2 && run g2f0 PBH_FAIR=0 PHASE_WORKLOAD=gmm2 && \
run g2h PBH_FAIR=0 PHASE_WORKLOAD=gmm2 PHASE_N=16384
