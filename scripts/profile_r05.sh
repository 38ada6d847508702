# rocprofv3 evidence for the headline bench at HEAD (run on the GPU box from
# the repo root).  Driver shape (--steps 20 --warmup 5): the timed run is a
# command to the resident server (PBH_SERVER=1, bench.py's default), so
#  * s20srv: the bench as the driver runs it -- kernel trace + stats (the
#    server kernel is one dispatch spanning the warm-up commands, the timed
#    command and the idle tail), the bench lines, the server's per-command
#    device stamps (scripts/server_probe.py);
#  * s20: the same 20 steps as an ordinary launch (PBH_SERVER=0: the same
#    step code, launched), for the per-launch kernel time and the FETCH_SIZE /
#    WRITE_SIZE / SQ passes the roofline's traffic is taken from;
#  * s1000: the default shape (1000 steps in 250-step launches, not a server
#    run), all passes.
# tools/collect_r05.py copies them into profiles/ with the library's sha256.
set -e
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/prof5
rm -rf $OUT && mkdir -p $OUT
sha256sum probayes_amd/libpbhip.so > $OUT/lib.sha256
cd /tmp
mkdir -p $OUT/s20srv
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/s20srv/trace -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-replay > $OUT/s20srv/bench_trace.log 2>&1
for i in 1 2 3; do timeout -k 10 200 python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-replay >> $OUT/s20srv/bench.log 2>&1; done
timeout -k 10 120 python3 $R/scripts/server_probe.py 65536 20 > $OUT/s20srv/probe.jsonl 2>&1
for S in s20 s1000; do
  mkdir -p $OUT/$S
  if [ $S = s20 ]; then ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-replay"; else ARGS="--steps 1000 --warmup 250 --no-cpu-baseline --no-replay"; fi
  export PBH_SERVER=0
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$S/trace -o run -- python3 $R/bench.py $ARGS > $OUT/$S/bench_trace.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$S/fetch -o run -- python3 $R/bench.py $ARGS > $OUT/$S/bench_fetch.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$S/write -o run -- python3 $R/bench.py $ARGS > $OUT/$S/bench_write.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $OUT/$S/sq -o run -- python3 $R/bench.py $ARGS > $OUT/$S/bench_sq.log 2>&1
  timeout -k 10 200 python3 $R/bench.py $ARGS > $OUT/$S/bench.log 2>&1
  unset PBH_SERVER
done
cd $R
timeout -k 10 300 python3 bench.py > $OUT/bench_default.log 2>&1
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1
