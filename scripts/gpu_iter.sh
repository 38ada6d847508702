# One iteration on the GPU: the -m gpu suite (stops at the first failure),
# then the headline evidence (scripts/gpu_headline.sh TAG).
# usage: bash scripts/gpu_iter.sh TAG [pytest selection]
export TMPDIR=/tmp
TAG=${1:-it}; shift
mkdir -p gpurun_out/$TAG
SEL=${@:-tests}
timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -q -rf -p no:warnings --timeout 120 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/$TAG/tests.log; exit 1; }
tail -3 gpurun_out/$TAG/tests.log
bash scripts/gpu_headline.sh $TAG
