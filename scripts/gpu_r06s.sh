# Round 6: the engine resource cache (buffers, streams of destroyed engines),
# and the pipelined fused REPLAY removed): the GPU suite, smoke, the server
# probe, cfg5 and both bench shapes.  usage: bash scripts/gpu_r06s.sh TAG
export TMPDIR=/tmp
TAG=${1:-r06s}
OUT=gpurun_out/$TAG
mkdir -p $OUT
sha256sum probayes_amd/libpbhip.so > $OUT/lib.sha256
T="python -u -m pytest -q -rf -p no:warnings --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_server.py > $OUT/tests_server.log 2>&1 || exit $?
timeout -k 10 600 $T -x tests -m gpu > $OUT/tests.log 2>&1 || exit $?
tail -1 $OUT/tests.log > $OUT/tests_summary.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 120 python scripts/server_probe.py 65536 20 > $OUT/probe.jsonl 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_workloads.py --no-cpu-baseline --only cfg5 > $OUT/cfg5.jsonl 2>&1 || exit $?
timeout -k 10 300 python bench.py > $OUT/bench_default.jsonl 2> $OUT/bench_default.err || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.jsonl 2> $OUT/bench_driver.err || exit $?
timeout -k 10 200 python scripts/facade_workload.py 65536 1000 3 250 > $OUT/facade_workload.jsonl 2>&1 || exit $?
timeout -k 10 200 python scripts/setup_probe.py > $OUT/setup_probe.jsonl 2>&1 || exit $?
