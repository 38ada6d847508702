# kernel trace of the fused REPLAY probe with the twist-ahead pass
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/ahead_prof
mkdir -p $OUT
R=$PWD
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/scripts/replay_fused_probe.py 65536 1000 250 fused > $OUT/probe.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $R/scripts/replay_fused_probe.py 65536 1000 250 fused > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $R/scripts/replay_fused_probe.py 65536 1000 250 fused > $OUT/write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d $OUT/sq -o run -- python3 $R/scripts/replay_fused_probe.py 65536 1000 250 fused > $OUT/sq.log 2>&1 || exit $?
