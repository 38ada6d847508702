# rocprofv3 evidence for the headline bench at HEAD (run on the GPU box from
# the repo root).  Round 6 adds the counter passes of the instance the
# driver's shape actually times: the resident-server kernel
# (mh_pair_kernel<..., FULL, SRV>), one dispatch for the server's life (the
# warm-up commands and the timed one); tools/collect_r06.py divides its bytes
# over the steps commanded in that life.  Per shape:
#  * s20srv: bench --steps 20 --warmup 5 as the driver runs it (server on):
#    kernel trace + stats, FETCH_SIZE, WRITE_SIZE, SQ passes, bench lines,
#    the per-command device stamps (scripts/server_probe.py);
#  * s20: the same 20 steps launched (PBH_SERVER=0): trace, FETCH, WRITE;
#  * s1000: the default shape (1000 steps in 250-step launches): all passes.
# Every GPU step runs under its own time limit; a step that times out or
# dies on a signal ends the script (exit status passed on).
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/prof6
rm -rf $OUT && mkdir -p $OUT
sha256sum probayes_amd/libpbhip.so > $OUT/lib.sha256
cd /tmp
step() {   # step <log> <timeout> <cmd...>: run, stop the script on a kill / fault
  local log=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $log 2>&1
  local rc=$?
  echo "rc=$rc $*" >> $OUT/steps.txt
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -gt 128 ]; then
    echo "stopping after rc=$rc" >> $OUT/steps.txt
    exit $rc
  fi
  return 0
}
BA="--no-cpu-baseline --no-replay --no-launched"
mkdir -p $OUT/s20srv
step $OUT/s20srv/bench_trace.log 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/s20srv/trace -o run -- python3 $R/bench.py --steps 20 --warmup 5 $BA
step $OUT/s20srv/bench_fetch.log 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/s20srv/fetch -o run -- python3 $R/bench.py --steps 20 --warmup 5 $BA
step $OUT/s20srv/bench_write.log 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/s20srv/write -o run -- python3 $R/bench.py --steps 20 --warmup 5 $BA
step $OUT/s20srv/bench_sq.log 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d $OUT/s20srv/sq -o run -- python3 $R/bench.py --steps 20 --warmup 5 $BA
for i in 1 2 3; do step $OUT/s20srv/bench_$i.log 200 python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-replay; done
step $OUT/s20srv/probe.jsonl 120 python3 $R/scripts/server_probe.py 65536 20
for S in s20 s1000; do
  mkdir -p $OUT/$S
  if [ $S = s20 ]; then ARGS="--steps 20 --warmup 5 $BA"; else ARGS="--steps 1000 --warmup 250 $BA"; fi
  export PBH_SERVER=0
  step $OUT/$S/bench_trace.log 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$S/trace -o run -- python3 $R/bench.py $ARGS
  step $OUT/$S/bench_fetch.log 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$S/fetch -o run -- python3 $R/bench.py $ARGS
  step $OUT/$S/bench_write.log 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$S/write -o run -- python3 $R/bench.py $ARGS
  step $OUT/$S/bench_sq.log 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d $OUT/$S/sq -o run -- python3 $R/bench.py $ARGS
  step $OUT/$S/bench.log 200 python3 $R/bench.py $ARGS
  unset PBH_SERVER
done
cd $R
step $OUT/bench_default.log 300 python3 bench.py
step $OUT/bench_driver.log 200 python3 bench.py --steps 20 --warmup 5
