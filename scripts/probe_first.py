#!/usr/bin/env python3
"""Wall time of the FIRST timed 20-step launch after a warm-up (the bench's
shape) versus the following ones, in one process; and with the first timed
launch preceded by a few empty syncs."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from probayes_amd import Engine  # noqa: E402

for variant in ('plain', 'spin'):
  eng = Engine(bench.cfg2_spec())
  eng.init_chains(np.zeros((65536, bench.D)))
  eng.set_rng('philox', seed=1)
  eng.set_collect(moments=False)
  eng.alloc_trace(5 + 20 * 8, 1)
  eng.run(5, steps_per_launch=1)
  eng.sync()
  walls, kern = [], []
  for rep in range(8):
    if variant == 'spin':
      t_end = time.perf_counter() + 200e-6     # keep the host busy 200 us
      while time.perf_counter() < t_end:
        pass
    t0 = time.perf_counter()
    eng.run(20, steps_per_launch=250, sync=False)
    eng.sync()
    walls.append((time.perf_counter() - t0) * 1e6)
    kern.append(eng.last_run_ms()[0] * 1e3)
  eng.close()
  print(json.dumps({'variant': variant, 'wall_us': [round(w, 1) for w in walls],
                    'kernel_us': [round(k, 1) for k in kern]}), flush=True)
