# One iteration on the GPU: the whole -m gpu suite, then the headline
# evidence (scripts/gpu_headline.sh TAG).  Ordinary test failures (pytest rc
# 1) still run the headline; a timeout, crash or abort ends the call.
# usage: bash scripts/gpu_iter.sh TAG [pytest selection]
export TMPDIR=/tmp
TAG=${1:-it}; shift
mkdir -p gpurun_out/$TAG
SEL=${@:-tests}
timeout -k 10 600 python -u -m pytest $SEL -m gpu -q -rf -p no:warnings --timeout 120 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1
rc=$?
tail -12 gpurun_out/$TAG/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended rc=$rc"; exit $rc; fi
bash scripts/gpu_headline.sh $TAG
