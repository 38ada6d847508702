#!/bin/bash
# PMC passes of the fused REPLAY kernel and the two-kernel form (one probe
# run covers both), then the resident server's 1-step command.
# usage: bash scripts/gpu_fused_pmc.sh <tag>
T=$1
R=$(pwd)
mkdir -p gpurun_out/$T
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY --output-format csv -d $R/gpurun_out/$T/sq -o run -- python3 $R/scripts/replay_fused_probe.py 65536 500 250 > $R/gpurun_out/$T/sq.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM --output-format csv -d $R/gpurun_out/$T/sq2 -o run -- python3 $R/scripts/replay_fused_probe.py 65536 500 250 > $R/gpurun_out/$T/sq2.log 2>&1 || exit $?
cd $R
timeout -k 10 120 python3 -u scripts/server_probe.py 65536 1 > gpurun_out/$T/server_1step.jsonl 2>&1 || exit $?
timeout -k 10 120 python3 -u scripts/server_probe.py 65536 20 > gpurun_out/$T/server_20step.jsonl 2>&1
