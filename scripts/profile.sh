# rocprofv3 passes for the bench kernel (run on the GPU box from the repo root).
# Pass 1: kernel trace + stats; passes 2/3: FETCH_SIZE and WRITE_SIZE alone
# (TCC slots: they cannot share a pass; MI355X_MICROARCH.md §rocprofv3).
set -e
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/prof
rm -rf $OUT && mkdir -p $OUT
ARGS="--steps 1000 --warmup 250 --steps-per-launch 250 --no-cpu-baseline"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py $ARGS > $OUT/bench_trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $R/bench.py $ARGS > $OUT/bench_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $R/bench.py $ARGS > $OUT/bench_write.log 2>&1
find $OUT -name "*.csv" | head -50
# Gibbs (cfg3) and the other workloads: kernel trace only
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/workloads -o run -- python3 $R/scripts/bench_workloads.py > $OUT/workloads.log 2>&1
