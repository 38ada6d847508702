#!/bin/bash
# FULL pair kernel: 4- vs 8-wave workgroups and the lockstep barrier
# (PBH_PAIR_WG, PBH_LOCKSTEP), phase stamps (probe build) + bench lines.
# usage: bash scripts/gpu_lockstep.sh TAG
set -o pipefail
T=${1:-ls}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {   # name, env...
  local name=$1; shift
  env "$@" PBHIP_LIB=probayes_amd/libpbhip_ph.so PHASE_RAW=gpurun_out/${T}_${name}_raw.npz \
    timeout -k 10 240 python3 -u scripts/phase_probe.py "${T}_$name" > gpurun_out/${T}_${name}.jsonl 2> gpurun_out/${T}_${name}.err
}
bl() {   # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> gpurun_out/${T}_${name}_s20.jsonl 2>> gpurun_out/${T}_bench.err &&
  env "$@" timeout -k 10 120 python3 bench.py --gpus 1 --steps 1000 --warmup 250 >> gpurun_out/${T}_${name}_s1000.jsonl 2>> gpurun_out/${T}_bench.err
}
run w256 PBH_FAIR=0 PBH_PAIR_WG=256 && run w512 PBH_FAIR=0 PBH_PAIR_WG=512 && \
run l1 PBH_FAIR=0 PBH_PAIR_WG=512 PBH_LOCKSTEP=1 && run l4 PBH_FAIR=0 PBH_PAIR_WG=512 PBH_LOCKSTEP=4 && \
run w256half PBH_FAIR=0 PBH_PAIR_WG=256 PHASE_N=32768 && \
bl w256 PBH_FAIR=0 PBH_PAIR_WG=256 && bl l1 PBH_FAIR=0 PBH_PAIR_WG=512 PBH_LOCKSTEP=1 && \
bl l4 PBH_FAIR=0 PBH_PAIR_WG=512 PBH_LOCKSTEP=4 && bl w256 PBH_FAIR=0 PBH_PAIR_WG=256 && \
bl l1 PBH_FAIR=0 PBH_PAIR_WG=512 PBH_LOCKSTEP=1
