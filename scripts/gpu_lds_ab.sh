# LDS bank-conflict A/B: the shipped library against a
# timing-only build whose table lookups read wave-uniform addresses
# (-DPBH_LDS_AB, probayes_amd/libpbhip_ab.so: no conflicts, wrong numbers),
# interleaved: 20-step driver-shape lines, 250-step lines, the cfg5 workload.
export TMPDIR=/tmp
T=${1:-ldsab}
mkdir -p gpurun_out/$T
for rep in 1 2 3; do
  for lib in libpbhip.so libpbhip_ab.so; do
    PBHIP_LIB=$PWD/probayes_amd/$lib timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-replay | sed "s/^/$lib s20 /" >> gpurun_out/$T/lines.txt || exit $?
    PBHIP_LIB=$PWD/probayes_amd/$lib timeout -k 10 120 python bench.py --steps 1000 --warmup 250 --no-cpu-baseline --no-replay | sed "s/^/$lib s1000 /" >> gpurun_out/$T/lines.txt || exit $?
  done
done
for lib in libpbhip.so libpbhip_ab.so libpbhip.so libpbhip_ab.so; do
  PBHIP_LIB=$PWD/probayes_amd/$lib timeout -k 10 200 python scripts/bench_workloads.py --only cfg5,cfg1 --no-cpu-baseline | sed "s/^/$lib /" >> gpurun_out/$T/workloads.txt || exit $?
done
cd /tmp
for lib in libpbhip.so libpbhip_ab.so; do
  PBHIP_LIB=$OLDPWD/probayes_amd/$lib timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_VALU --output-format csv -d $OLDPWD/gpurun_out/$T/pmc_$lib -o run -- python3 $OLDPWD/bench.py --steps 1000 --warmup 250 --no-cpu-baseline --no-replay > $OLDPWD/gpurun_out/$T/pmc_$lib.log 2>&1 || exit $?
done
