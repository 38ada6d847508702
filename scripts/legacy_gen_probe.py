#!/usr/bin/env python3
"""Device legacy stream generation (pbh_legacy_replay) for the forms the
fused kernel does not cover, timed per launch: gibbs8 (cfg3's CondCov
rows, the chain-per-lane Mt4 generator) at 32 768 chains x 256 steps.
PBH_LEGACY_AHEAD (read at engine creation) switches the twist-ahead pass.
One JSON line per form.  usage: legacy_gen_probe.py [chains] [steps] [reps]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402  (the golden workload's spec only)
from probayes_amd import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 256
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
for name in ['gibbs8']:
  spec = oracle.golden_spec(name)
  eng = Engine(spec)
  eng.init_chains(np.zeros((n, spec['dim'])))
  eng.set_rng('replay')
  eng.seed_legacy(np.arange(n))
  eng.legacy_replay(steps)   # warm-up (allocations)
  eng.sync()
  t0 = time.perf_counter()
  for _ in range(reps):
    eng.legacy_replay(steps)
  el = (time.perf_counter() - t0) / reps
  print(json.dumps({'workload': name, 'chains': n, 'steps': steps,
                    'ahead': os.environ.get('PBH_LEGACY_AHEAD', '1'),
                    'ms_per_generation': el * 1e3}), flush=True)
  eng.close()
