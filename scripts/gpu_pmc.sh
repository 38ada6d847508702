set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 tools/ubench/ubench > gpurun_out/ubench.log 2>&1 || exit 1
timeout -k 10 600 bash scripts/pmc_pair.sh || exit 1
for d in gpurun_out/pmc/*/; do find $d -name "*counter_collection.csv" | head -1 | xargs -I{} python3 -c "
import csv,sys,collections
rows=list(csv.DictReader(open('{}')))
agg=collections.defaultdict(float); n=collections.Counter()
for r in rows:
  if 'mh_pair' in r['Kernel_Name']:
    agg[r['Counter_Name']]+=float(r['Counter_Value']); n[r['Counter_Name']]+=1
print({k:(v/ (n[k]) ) for k,v in agg.items()}, dict(n))
" ; done > gpurun_out/pmc_summary.log 2>&1
