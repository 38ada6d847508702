#!/usr/bin/env python3
"""Timing events on the dispatch packet (default) vs marker packets
(PBH_EVENT_MARKERS=1): kernel and wall time of short cfg2 launches, and of a
one-wave launch (the fixed dispatch cost)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'scripts'))
from launch_probe import probe  # noqa: E402

if __name__ == '__main__':
  for markers in ('0', '1'):
    os.environ['PBH_EVENT_MARKERS'] = markers
    print('markers', markers, flush=True)
    for chains, steps in ((64, 1), (65536, 1), (65536, 20), (65536, 250)):
      probe('philox', False, steps, 20 if steps < 250 else 6, None,
            trace=True, chains=chains)
