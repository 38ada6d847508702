#!/bin/bash
# Phase stamps of the FULL pair kernel (probe build) + kernel trace of the same.
# usage: bash scripts/gpu_phase.sh TAG
set -o pipefail
T=${1:-ph}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PBHIP_LIB=probayes_amd/libpbhip_ph.so PHASE_RAW=gpurun_out/${T}_phase_raw.npz timeout -k 10 240 python3 -u scripts/phase_probe.py "$T" > gpurun_out/${T}_phase.jsonl 2> gpurun_out/${T}_phase.err
