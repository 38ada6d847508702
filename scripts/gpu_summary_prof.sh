export TMPDIR=/tmp
mkdir -p gpurun_out/summary
timeout -k 10 300 python scripts/summary_profile.py > gpurun_out/summary/profile.txt 2>&1 || exit $?
