# Round 6: the pipelined fused REPLAY (producer / consumer waves) -- its
# parity tests and the A/B probe against the single-wave fused kernel; the
# server command protocols (tools/ubench/mailbox_rtt, then the engine's
# PBH_SERVER_DIRECT / PBH_SERVER_SINGLE: server tests and driver-shape bench
# lines); then the GPU suite, smoke and both bench shapes.
# usage: bash scripts/gpu_r06p.sh TAG
export TMPDIR=/tmp
TAG=${1:-r06p}
OUT=gpurun_out/$TAG
mkdir -p $OUT
sha256sum probayes_amd/libpbhip.so > $OUT/lib.sha256
T="python -u -m pytest -q -rf -p no:warnings --timeout 120 --timeout-method thread"
timeout -k 10 300 env PBH_LEGACY_PIPE=1 $T tests/test_gpu_legacy_fused.py tests/test_gpu_parity.py -k "fused or replay or legacy" > $OUT/tests_fused.log 2>&1 || exit $?
for i in 1 2; do
timeout -k 10 120 env PBH_LEGACY_PIPE=1 python scripts/replay_fused_probe.py 65536 1000 250 fused >> $OUT/probe_pipe.jsonl 2>&1 || exit $?
timeout -k 10 120 env PBH_LEGACY_PIPE=0 python scripts/replay_fused_probe.py 65536 1000 250 fused >> $OUT/probe_single.jsonl 2>&1 || exit $?
done
for m in 0 1 2 3; do
timeout -k 10 60 tools/ubench/bin/mailbox_rtt $m 3000 20 256 >> $OUT/mailbox_rtt.jsonl 2>&1
rc=$?; echo "mode $m rc=$rc" >> $OUT/mailbox_rtt.jsonl
if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done
timeout -k 10 300 env PBH_SERVER_DIRECT=1 PBH_SERVER_SINGLE=1 $T tests/test_gpu_server.py > $OUT/tests_server_ds.log 2>&1 || exit $?
for i in 1 2; do
for v in "0 0" "0 1" "1 0" "1 1"; do
set -- $v
timeout -k 10 200 env PBH_SERVER_DIRECT=$1 PBH_SERVER_SINGLE=$2 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-replay --no-launched > $OUT/s20_d$1s$2_$i.jsonl 2>&1 || exit $?
done
done
timeout -k 10 600 $T tests -m gpu > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $OUT/bench_default.jsonl 2> $OUT/bench_default.err || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.jsonl 2> $OUT/bench_driver.err || exit $?
