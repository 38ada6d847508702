export TMPDIR=/tmp
mkdir -p gpurun_out/r04ae
for r in 1 2; do
for cfg in "k11:" "k10:PBH_FAIR=10" "k12:PBH_FAIR=12" "k9:PBH_FAIR=9" "rel11:PBH_FAIR_REL=1" "off:PBH_FAIR=0"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  echo -n "$name " >> gpurun_out/r04ae/c5.txt
  env $envs timeout -k 10 60 python3 scripts/cfg5_kernel.py >> gpurun_out/r04ae/c5.txt 2>&1 || exit $?
done
done
