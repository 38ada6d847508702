set -o pipefail
for a in "" "--no-trace" "--rng xoshiro" "--rng xoshiro --no-trace" "--chains 131072" ""; do
  timeout -k 10 120 python bench.py --no-cpu-baseline $a | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print('$a', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])" || exit 1
done
