#!/usr/bin/env python3
"""One device legacy-stream workload (cfg2 width, polar normals or uniforms)
for rocprofv3 passes: seed, then 3 generation launches of 250 steps."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
from probayes_amd import Engine  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else 'gauss'
n, t = 65536, 250
spec = oracle.golden_spec('diag10')
if kind == 'uniform':
  spec['proposal'] = {'kind': 'uniform', 'delta': np.full(10, 0.3)}
eng = Engine(spec)
eng.init_chains(np.zeros((n, 10)))
eng.seed_legacy(np.arange(n))
for _ in range(3):
  eng.legacy_replay(t)
eng.close()
