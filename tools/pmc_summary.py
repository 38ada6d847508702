#!/usr/bin/env python3
"""Per-dispatch averages of rocprofv3 --pmc counter_collection.csv files,
per kernel (name filter optional).  usage: pmc_summary.py <dir> [substr]"""
import collections
import csv
import glob
import sys

root = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ''
for f in sorted(glob.glob(root + '/**/*counter_collection.csv', recursive=True)):
  agg = collections.defaultdict(lambda: collections.defaultdict(float))
  cnt = collections.Counter()
  for r in csv.DictReader(open(f)):
    k = r['Kernel_Name']
    if sub not in k:
      continue
    agg[k][r['Counter_Name']] += float(r['Counter_Value'])
    cnt[(k, r['Counter_Name'])] += 1
  print('==', f)
  for k, v in agg.items():
    avg = {c: x / max(1, cnt[(k, c)]) for c, x in v.items()}
    line = {c: '{:.4g}'.format(x) for c, x in avg.items()}
    wc = avg.get('SQ_WAVE_CYCLES')
    if wc:
      for c in ('SQ_WAIT_INST_ANY', 'SQ_WAIT_ANY', 'SQ_ACTIVE_INST_VALU'):
        if c in avg:
          line[c + '/WAVE_CYCLES'] = '{:.3f}'.format(avg[c] / wc)
    print(k[:90], line)
