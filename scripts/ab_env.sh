# A/B of engine environment knobs on one box: bench lines at the driver's
# shape (--steps 20 --warmup 5) and at 250-step launches, rounds interleaved.
# usage: bash scripts/ab_env.sh TAG ROUNDS "name1:VAR=v VAR=v" "name2:..." ...
export TMPDIR=/tmp
TAG=$1; R=$2; shift 2
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for cfg in "$@"; do
    name=${cfg%%:*}; envs=${cfg#*:}
    env $envs timeout -k 10 60 python bench.py --steps 20 --warmup 5 --no-cpu-baseline | sed "s/^{/{\"ab\": \"$name\", \"shape\": \"s20\", /" >> gpurun_out/${TAG}_ab.jsonl || exit $?
  done
done
for cfg in "$@"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 100 python bench.py --steps 1000 --warmup 250 --no-cpu-baseline | sed "s/^{/{\"ab\": \"$name\", \"shape\": \"s1000\", /" >> gpurun_out/${TAG}_ab.jsonl || exit $?
done
