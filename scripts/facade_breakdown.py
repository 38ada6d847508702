#!/usr/bin/env python3
"""Where the seeded facade sampler's walk spends its time outside the
kernels: every Engine method the sampler calls is wrapped with a timer (host
wall, ms, summed per method), around one 65 536-chain x 1 000-step walk of
the diag10 example (after a warm-up walk).  One JSON line per repetition."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import probayes_amd as pb  # noqa: E402
from probayes_amd import engine as E  # noqa: E402
from mcmc_examples import WORKLOADS  # noqa: E402

acc = {}


def wrap(name):
  f = getattr(E.Engine, name)

  def g(*a, **k):
    t = time.perf_counter()
    try:
      return f(*a, **k)
    finally:
      acc[name] = acc.get(name, 0.0) + (time.perf_counter() - t) * 1e3
  setattr(E.Engine, name, g)


for m in ['__init__', 'init_chains', 'set_rng', 'seed_legacy', 'set_record_threshold',
          'alloc_trace', 'legacy_run', 'sync', 'state', 'set_step']:
  if hasattr(E.Engine, m):
    wrap(m)
from probayes_amd import sp as S  # noqa: E402


def wrap_s(name):
  f = getattr(S.Sampler, name)

  def g(*a, **k):
    t = time.perf_counter()
    try:
      return f(*a, **k)
    finally:
      acc['Sampler.' + name] = acc.get('Sampler.' + name, 0.0) + (time.perf_counter() - t) * 1e3
  setattr(S.Sampler, name, g)


for m in ['_lower', '_init_array', '_start_epoch', '_compute']:
  wrap_s(m)
n, T, spl = 65536, 1000, 250
builder, params, _, _, _ = WORKLOADS['diag10']
process, init, extra, kwds, keys = builder(pb, params)
args = (init,) if extra is None else (init, extra)
seeds = np.arange(n) + 12345
for rep in range(4):
  acc.clear()
  t0 = time.perf_counter()
  sm = process.sampler(*args, stop=T, chains=n, seeds=seeds, steps_per_launch=spl, **kwds)
  t1 = time.perf_counter()
  it = iter(sm)
  first = next(it)
  t2 = time.perf_counter()
  rest = list(it)
  t3 = time.perf_counter()
  sm.close()
  if rep:
    print(json.dumps({'sampler_ms': (t1 - t0) * 1e3, 'first_ms': (t2 - t1) * 1e3,
                      'rest_ms': (t3 - t2) * 1e3, 'walk_ms': (t3 - t0) * 1e3,
                      'engine_ms': {k: round(v, 3) for k, v in acc.items()}}), flush=True)
