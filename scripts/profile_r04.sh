# rocprofv3 evidence for the headline bench at HEAD (run on the GPU box from
# the repo root): for the driver's shape (--steps 20 --warmup 5: one 20-step
# timed launch) and the default shape (1000 steps in 250-step launches), a
# kernel trace + stats pass, separate FETCH_SIZE / WRITE_SIZE passes and one
# SQ pass; the bench JSON lines themselves.  tools/collect_profiles.py copies
# them into profiles/ with the library's sha256.
set -e
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/prof4
rm -rf $OUT && mkdir -p $OUT
sha256sum probayes_amd/libpbhip.so > $OUT/lib.sha256
cd /tmp
for S in s20 s1000; do
  mkdir -p $OUT/$S
  if [ $S = s20 ]; then ARGS="--steps 20 --warmup 5 --no-cpu-baseline"; else ARGS="--steps 1000 --warmup 250 --no-cpu-baseline"; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$S/trace -o run -- python3 $R/bench.py $ARGS > $OUT/$S/bench_trace.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$S/fetch -o run -- python3 $R/bench.py $ARGS > $OUT/$S/bench_fetch.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$S/write -o run -- python3 $R/bench.py $ARGS > $OUT/$S/bench_write.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $OUT/$S/sq -o run -- python3 $R/bench.py $ARGS > $OUT/$S/bench_sq.log 2>&1
  timeout -k 10 200 python3 $R/bench.py $ARGS > $OUT/$S/bench.log 2>&1
done
cd $R
timeout -k 10 300 python3 bench.py > $OUT/bench_default.log 2>&1
