#!/usr/bin/env python3
"""The seeded (reference-identical) SP sampler end to end through the façade
at cfg2 width: the diag10 example model
(tests/mcmc_examples.py, the cfg2 target and callable Gaussian Delta) as
SP.sampler(init, stop=T, chains=65536, seeds=...) + SP.walk, then the
summary.  One JSON line per repetition:
  walk_s     -- sampler + walk: the engine run (pbh_legacy_run, the fused
                REPLAY kernel with the device RandomStates) and the T Step
                objects; the trace stays on the device;
  summary_s  -- SP(samples): the trace copied to the host and the PDs built;
  chain_steps_per_s -- N T / walk_s, beside bench.py's replay_chain_steps_per_s.
usage: facade_workload.py [chains] [steps] [reps] [steps_per_launch] [walk|iter]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import probayes_amd as pb  # noqa: E402
from mcmc_examples import WORKLOADS  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
T = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
spl = int(sys.argv[4]) if len(sys.argv) > 4 else 250   # bench.py's REPLAY launches
walk = (sys.argv[5] if len(sys.argv) > 5 else 'walk') == 'walk'   # or 'iter': next() per step
builder, params, _, _, _ = WORKLOADS['diag10']
process, init, extra, kwds, keys = builder(pb, params)
args = (init,) if extra is None else (init, extra)
seeds = np.arange(n) + 12345
for rep in range(reps + 1):   # the first is a warm-up (library load, allocations)
  t0 = time.perf_counter()
  sm = process.sampler(*args, stop=T, chains=n, seeds=seeds,
                       steps_per_launch=spl, **kwds)
  if walk:   # SP.walk, as examples/mcmc consume a sampler
    samples = process.walk(sm)
    tf = t1 = time.perf_counter()
  else:
    it = iter(sm)
    first = next(it)            # the engine run: all T steps
    tf = time.perf_counter()
    samples = [first] + list(it)
    t1 = time.perf_counter()
  summary = process(samples)
  t2 = time.perf_counter()
  assert np.asarray(summary.v[keys[0]]).shape == (T, n)
  sm.close()
  if rep:
    print(json.dumps({'workload': 'facade seeded diag10 (cfg2 shape)', 'chains': n,
                      'consumed_by': 'SP.walk' if walk else 'next() per step',
                      'steps': T, 'steps_per_launch': spl, 'walk_s': t1 - t0,
                      'first_step_s': None if walk else tf - t0,
                      'other_steps_s': None if walk else t1 - tf,
                      'summary_s': t2 - t1,
                      'chain_steps_per_s': n * T / (t1 - t0),
                      'end_to_end_chain_steps_per_s': n * T / (t2 - t0)}), flush=True)
