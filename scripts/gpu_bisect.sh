# one failing façade test on two trees: A (the previous commit, in bisectA/)
# then B (the working tree); stops at the first failure
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/bisect
mkdir -p $OUT
T="python -u -m pytest -x -q -p no:warnings --timeout 120 --timeout-method thread"
K="tests/test_facade.py::test_batched_sampler_reproduces_all_reference_chains"
(cd bisectA && timeout -k 10 200 $T "$K[metrohast_norm1d]" "$K[diag10]" > $OUT/A.log 2>&1) || exit $?
timeout -k 10 200 env HIP_LAUNCH_BLOCKING=1 AMD_SERIALIZE_KERNEL=3 $T "$K[metrohast_norm1d]" "$K[diag10]" > $OUT/B.log 2>&1 || exit $?
