#!/usr/bin/env python3
"""Median value / events / enqueue per (ab, shape) of an ab_env.sh file."""
import collections, json, sys
import numpy as np
rows = collections.defaultdict(list)
for line in open(sys.argv[1]):
  if line.startswith('{'):
    d = json.loads(line)
    rows[(d['ab'], d['shape'])].append(d)
for (ab, sh), ds in sorted(rows.items(), key=lambda kv: (kv[0][1], kv[0][0])):
  v = np.array([d['value'] for d in ds])
  ev = np.array([d['events_us'] for d in ds])
  enq = np.array([d['host_enqueue_us'] for d in ds])
  wall = np.array([d['ms_per_step'] * d['steps'] * 1e3 for d in ds])
  print('{:6s} {:10s} n={:2d} value med {:.3e} (min {:.3e} max {:.3e})  events {:.1f}  enq {:.1f}  wall {:.1f} us  frac {:.3f}'.format(
      sh, ab, len(ds), np.median(v), v.min(), v.max(), np.median(ev), np.median(enq),
      np.median(wall), np.median([d['roofline']['frac'] for d in ds])))
