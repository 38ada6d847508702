#!/bin/bash
# Phase stamps of the FULL pair kernel (probe build), one run per knob set.
# usage: bash scripts/gpu_phase.sh TAG "name:VAR=v VAR=v" ...
set -o pipefail
T=${1:-ph}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "$@"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs PBHIP_LIB=probayes_amd/libpbhip_ph.so PHASE_RAW=gpurun_out/${T}_${name}_phase_raw.npz timeout -k 10 240 python3 -u scripts/phase_probe.py "$name" >> gpurun_out/${T}_phase.jsonl 2>> gpurun_out/${T}_phase.err || exit $?
done
