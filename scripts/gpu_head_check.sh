#!/bin/bash
# HEAD check: driver-shape bench lines, the default bench and the workload lines.
set -o pipefail
T=${1:-hc}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2 3; do
  timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> gpurun_out/${T}_s20.jsonl 2>> gpurun_out/${T}_bench.err || exit $?
done
timeout -k 10 180 python3 bench.py >> gpurun_out/${T}_default.jsonl 2>> gpurun_out/${T}_bench.err &&
timeout -k 10 300 python3 scripts/bench_workloads.py > gpurun_out/${T}_wl.jsonl 2> gpurun_out/${T}_wl.err
