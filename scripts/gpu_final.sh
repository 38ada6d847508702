# Round-end evidence at HEAD: GPU suite, smoke, workloads, the rocprofv3
# passes of the headline at the driver's and the default shape (with the
# bench lines), and the legacy generator's passes
export TMPDIR=/tmp
TAG=${1:-fin}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -rf -p no:warnings --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_workloads.py --no-cpu-baseline > gpurun_out/${TAG}_wl.jsonl 2>&1 || exit $?
bash scripts/profile_r04.sh || exit $?
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 >> gpurun_out/${TAG}_s20_lines.jsonl 2>&1 || exit $?
done
bash scripts/gpu_legacy_pmc.sh ${TAG}_leg
