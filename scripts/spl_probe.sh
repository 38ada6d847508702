set -o pipefail
for spl in 250 500 1000 125; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 1000 --warmup 1000 --steps-per-launch $spl | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print('spl $spl', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['ms_per_step'])" || exit 1
done
