# the GPU suite and smoke at HEAD.  usage: bash scripts/gpu_suite.sh TAG
export TMPDIR=/tmp
OUT=gpurun_out/${1:-suite}
mkdir -p $OUT
sha256sum probayes_amd/libpbhip.so > $OUT/lib.sha256
timeout -k 10 500 python -u -m pytest tests -m gpu -q -rf -p no:warnings --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit $?
tail -1 $OUT/tests.log > $OUT/tests_summary.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
