"""Per-kernel averages of the PMC passes written by gpu_pmc_kernel.sh, plus
derived per-wave-step figures.  usage: pmc_summary.py <dir> [kernel-substr]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ''
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(d + '/p*/**/*counter_collection.csv', recursive=True):
  for r in csv.DictReader(open(f)):
    if sub in r['Kernel_Name']:
      agg[r['Kernel_Name']][r['Counter_Name']].append(float(r['Counter_Value']))
for k, cs in agg.items():
  print(k[:90])
  for c, v in sorted(cs.items()):
    print('  {:24s} max {:16.1f}  mean {:16.1f} (n={})'.format(c, max(v), sum(v) / len(v), len(v)))
