# cfg5 quad kernel A/B: the quad parity tests, then interleaved kernel times
# of the current library and libpbhip_ab.so (a reference build), then a SQ
# PMC pass of the current one.  usage: bash scripts/gpu_cfg5_ab.sh TAG [ROUNDS]
export TMPDIR=/tmp
R=$PWD; T=${1:-c5ab}; N=${2:-3}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:warnings --timeout 120 --timeout-method thread -k "gmm or ess" > gpurun_out/$T/tests.log 2>&1 || exit $?
for r in $(seq 1 $N); do
  for lib in libpbhip.so libpbhip_ab.so; do
    PBHIP_LIB=$R/probayes_amd/$lib timeout -k 10 60 python3 scripts/cfg5_kernel.py | sed "s/^/$lib /" >> gpurun_out/$T/times.txt 2>&1 || exit $?
  done
done
cd /tmp
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY --output-format csv -d $R/gpurun_out/$T/sq -o run -- python3 $R/scripts/cfg5_kernel.py > $R/gpurun_out/$T/sq.log 2>&1
