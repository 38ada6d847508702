# Resident server A/B: the server GPU tests on the current library, then
# interleaved server probes and driver-shape bench lines of the current
# library and libpbhip_ab.so.  usage: bash scripts/gpu_srv_ab.sh TAG [ROUNDS]
export TMPDIR=/tmp
R=$PWD; T=${1:-srvab}; N=${2:-3}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_server.py -x -q -p no:warnings --timeout 120 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || exit $?
for r in $(seq 1 $N); do
  for lib in libpbhip.so libpbhip_ab.so; do
    PBHIP_LIB=$R/probayes_amd/$lib timeout -k 10 120 python3 scripts/server_probe.py 65536 20 | sed "s/^{/{\"lib\": \"$lib\", /" >> gpurun_out/$T/probe.jsonl 2>&1 || exit $?
    PBHIP_LIB=$R/probayes_amd/$lib timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-replay | sed "s/^{/{\"lib\": \"$lib\", /" >> gpurun_out/$T/bench.jsonl 2>&1 || exit $?
  done
done
