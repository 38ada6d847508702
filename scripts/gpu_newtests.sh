export TMPDIR=/tmp
mkdir -p gpurun_out/newtests
timeout -k 10 300 python -u -m pytest -q -rf -p no:warnings --timeout 120 --timeout-method thread tests/test_facade.py -k "walk_hands_out or cached_buffers or batched" > gpurun_out/newtests/tests.log 2>&1 || exit $?
