# Quick GPU iteration: the given pytest targets, then the workload bench.
# usage: bash scripts/gpu_iter.sh "<pytest targets>" [extra step command]
export TMPDIR=/tmp
O=$PWD/gpurun_out
mkdir -p $O
rm -f $O/iter_*.log
timeout -k 10 400 python -u -m pytest $1 -x -q -rf -p no:warnings --timeout 120 --timeout-method thread > $O/iter_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/iter_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 240 python scripts/bench_workloads.py > $O/iter_workloads.log 2>&1 || exit $?
if [ -n "$2" ]; then timeout -k 10 300 bash -c "$2" > $O/iter_extra.log 2>&1 || exit $?; fi
echo ok
