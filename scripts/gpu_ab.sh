export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in $2 $3; do
    timeout -k 10 120 python scripts/bench_ab.py $v --no-cpu-baseline | sed "s|^|$v |" >> gpurun_out/${1}_ab.txt || exit $?
  done
done
