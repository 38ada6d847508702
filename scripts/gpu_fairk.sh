#!/bin/bash
# Wave-priority alternation period sweep (PBH_FAIR=k: 2^k x 10 ns) on the
# FULL pair and quad kernels: phase stamps + bench lines.  usage: gpu_fairk.sh TAG
set -o pipefail
T=${1:-fk}
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
run k0 PBH_FAIR=0 && run k9 PBH_FAIR=9 && run k11 PBH_FAIR=11 && run k13 PBH_FAIR=13 && \
run gk0 PBH_FAIR=0 PHASE_WORKLOAD=gmm2 && run gk11 PBH_FAIR=11 PHASE_WORKLOAD=gmm2 && \
bl k0 PBH_FAIR=0 && bl k9 PBH_FAIR=9 && bl k11 PBH_FAIR=11 && bl k0 PBH_FAIR=0 && bl k9 PBH_FAIR=9 && bl k11 PBH_FAIR=11
