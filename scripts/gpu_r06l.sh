# pipelined server polling + pbh_run_wait + ESS total: their suites, the
# server probe, the driver-shape bench lines, cfg5 workload
export TMPDIR=/tmp
TAG=${1:-r06l}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 120 python -u scripts/facade_profile.py > $OUT/facade_profile.txt 2>&1 || exit $?
true
true
timeout -k 10 300 python scripts/bench_workloads.py --no-cpu-baseline --only cfg5 > $OUT/cfg5.jsonl 2>&1 || exit $?
