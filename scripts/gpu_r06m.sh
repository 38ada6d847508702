# Round-6 state check at HEAD: GPU suite, smoke, default + driver-shape bench
export TMPDIR=/tmp
TAG=${1:-r06m}
OUT=gpurun_out/$TAG
mkdir -p $OUT
sha256sum probayes_amd/libpbhip.so > $OUT/lib.sha256
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -p no:warnings --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $OUT/bench_default.jsonl 2> $OUT/bench_default.err || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.jsonl 2> $OUT/bench_driver.err || exit $?
