#!/usr/bin/env python3
"""Device legacy-stream generation time (pbh_legacy_replay) at cfg2 width:
normals (polar rejection: lanes drift apart) vs uniforms (lanes in step),
65 536 chains x 250 steps."""
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
for db, kind in (('1', 'gauss'), ('1', 'uniform'), ('0', 'gauss'), ('0', 'uniform')):
  os.environ['PBH_LEGACY_DB'] = db
  spec = oracle.golden_spec('diag10')
  if kind == 'uniform':
    spec['proposal'] = {'kind': 'uniform', 'delta': np.full(10, 0.3)}
  eng = Engine(spec)
  eng.init_chains(np.zeros((n, 10)))
  eng.seed_legacy(np.arange(n))
  eng.legacy_replay(t)            # first call: includes the seeding twist
  times = []
  for _ in range(3):
    t0 = time.perf_counter()
    eng.legacy_replay(t)
    times.append((time.perf_counter() - t0) * 1e3)
  eng.close()
  print(json.dumps({'db': db, 'kind': kind, 'chains': n, 'steps': t, 'ms': times}), flush=True)
