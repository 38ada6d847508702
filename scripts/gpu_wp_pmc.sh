# PMC passes + store-free A/B of the word-parallel legacy generator
export TMPDIR=/tmp
TAG=${1:-r06c}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
for lib in libpbhip.so libpbhip_wpns.so libpbhip.so libpbhip_wpns.so; do
  PBHIP_LIB=$R/probayes_amd/$lib timeout -k 10 60 python3 scripts/legacy_kernel.py | sed "s/^/$lib /" >> $OUT/times.txt 2>&1 || exit $?
done
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $OUT/sq1 -o run -- python3 $R/scripts/legacy_kernel.py > $OUT/sq1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --output-format csv -d $OUT/sq2 -o run -- python3 $R/scripts/legacy_kernel.py > $OUT/sq2.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $R/scripts/legacy_kernel.py > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $R/scripts/legacy_kernel.py > $OUT/write.log 2>&1 || exit $?
