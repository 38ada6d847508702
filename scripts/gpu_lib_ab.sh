# Interleaved kernel timings of several library builds on one box.
# usage: bash scripts/gpu_lib_ab.sh TAG ROUNDS SCRIPT lib1.so lib2.so ...
# (SCRIPT prints one timing line; each line is prefixed with the library)
export TMPDIR=/tmp
R=$PWD; T=$1; N=$2; S=$3; shift 3
mkdir -p gpurun_out/$T
for r in $(seq 1 $N); do
  for lib in "$@"; do
    PBHIP_LIB=$R/probayes_amd/$lib timeout -k 10 60 python3 $S | sed "s/^/$lib /" >> gpurun_out/$T/times.txt 2>&1 || exit $?
  done
done
