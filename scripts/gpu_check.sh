# GPU suite + smoke + headline bench lines (driver shape x3, default x1).
# usage: bash scripts/gpu_check.sh TAG [pytest selection...]
export TMPDIR=/tmp
TAG=${1:-chk}; shift
SEL=${@:-tests}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest $SEL -m gpu -q -rf -p no:warnings --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> gpurun_out/${TAG}_s20.jsonl 2>&1 || exit $?
done
timeout -k 10 200 python bench.py --no-cpu-baseline >> gpurun_out/${TAG}_default.jsonl 2>&1 || exit $?
