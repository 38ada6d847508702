T=esslg
mkdir -p gpurun_out/$T
PBHIP_LIB=$PWD/probayes_amd/libpbhip_lg.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "ess" > gpurun_out/$T/tests.log 2>&1 || exit $?
for r in 1 2 3; do for lib in libpbhip.so libpbhip_lg.so; do
  PBHIP_LIB=$PWD/probayes_amd/$lib timeout -k 10 120 python -u scripts/ess_call_probe.py | sed "s/^/$lib /" >> gpurun_out/$T/probe.txt || exit $?
done; done
cd /tmp && export TMPDIR=/tmp
for lib in libpbhip.so libpbhip_lg.so; do
  PBHIP_LIB=$OLDPWD/probayes_amd/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OLDPWD/gpurun_out/$T/kt_$lib -o run -- python3 $OLDPWD/scripts/ess_call_probe.py > $OLDPWD/gpurun_out/$T/kt_$lib.log 2>&1 || exit $?
done
