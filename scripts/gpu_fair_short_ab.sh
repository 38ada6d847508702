export TMPDIR=/tmp
mkdir -p gpurun_out/s1fair
for r in 1 2 3; do
  for cfg in "k10:PBH_FAIR_SHORT=10" "k9:PBH_FAIR_SHORT=9" "k11:PBH_FAIR_SHORT=11" "k8:PBH_FAIR_SHORT=8"; do
    name=${cfg%%:*}; envs=${cfg#*:}
    env $envs timeout -k 10 120 python3 scripts/server_probe.py 65536 20 | sed "s/^{/{\"ab\": \"$name\", /" >> gpurun_out/s1fair/probe.jsonl || exit $?
  done
done
