#!/usr/bin/env python3
"""Device legacy-stream generation alone (for PMC passes): cfg2 width
(65 536 chains x 10 polar normals + the threshold), 250 steps, after a
first call that includes the seeding twist."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
from probayes_amd import Engine  # noqa: E402

n, t = 65536, 250
eng = Engine(oracle.golden_spec('diag10'))
eng.init_chains(np.zeros((n, 10)))
eng.seed_legacy(np.arange(n))
eng.legacy_replay(t)
times = []
for _ in range(3):
  t0 = time.perf_counter()
  eng.legacy_replay(t)
  times.append((time.perf_counter() - t0) * 1e3)
eng.close()
print(json.dumps({'kind': 'gauss', 'chains': n, 'steps': t, 'wall_ms': times}), flush=True)
