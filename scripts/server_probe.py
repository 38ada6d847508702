#!/usr/bin/env python3
"""Resident-server command timing at the driver's shape (cfg2, 65 536 chains,
20-step commands after a 5-step warm-up): per command the host wall time,
the device span (first workgroup's sight to last completion), the spread of
the workgroups' sights and of their completion times."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault('PBH_SERVER', '1')
os.environ.setdefault('PBH_SPIN_FLAG', '1')
import bench  # noqa: E402
from probayes_amd import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
eng = Engine(bench.cfg2_spec())
eng.init_chains(np.zeros((n, bench.D)))
eng.set_rng('philox', seed=7)
eng.set_collect(moments=False)
eng.alloc_trace(5 + 12 * steps, 1)
for _ in range(5):
  eng.run(1)
for rep in range(10):
  t0 = time.perf_counter()
  eng.run(steps)   # pbh_run_wait: one call
  wall = (time.perf_counter() - t0) * 1e6
  ms, _ = eng.last_run_ms()
  q, a, b = eng.server_stamps()
  a = a.astype(np.int64)
  b = b.astype(np.int64)
  print(json.dumps({'n': n, 'steps': steps, 'wall_us': round(wall, 2),
                    'span_us': round(ms * 1e3, 2),
                    'sight_spread_us': float(a.max() - a.min()) / 100,
                    'done_spread_us': float(b.max() - b.min()) / 100,
                    'wg_dur_us_min_med_max': [float(np.min(b - a)) / 100,
                                              float(np.median(b - a)) / 100,
                                              float(np.max(b - a)) / 100],
                    'info': eng.server_info()}), flush=True)
eng.close()
