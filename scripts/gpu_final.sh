# Round-end evidence at HEAD: GPU suite, smoke, workloads, bench lines, and
# the rocprofv3 passes of the headline at the driver's and the default shape
export TMPDIR=/tmp
TAG=${1:-fin}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -rf -p no:warnings --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_workloads.py --no-cpu-baseline > gpurun_out/${TAG}_wl.jsonl 2>&1 || exit $?
bash scripts/profile_r03.sh || exit $?
bash scripts/gpu_legacy_prof.sh || exit $?
bash scripts/gpu_headline.sh ${TAG}_hl || exit $?
