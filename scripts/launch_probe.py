#!/usr/bin/env python3
"""Where the time of a short timed region goes (cfg2, 65 536 chains): per
variant, the median over repetitions of the wall time of run(K) + sync, the
host time of the enqueue alone, and the kernel time from the engine's HIP
events.  Variants: RNG mode, moments on/off, sync mode (PBH_SYNC), trace."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from probayes_amd import Engine  # noqa: E402


def probe(rng, moments, steps, reps, sync_env, trace=True, chains=65536,
          spl=250, tag=None):
  if sync_env:
    os.environ['PBH_SYNC'] = sync_env
  else:
    os.environ.pop('PBH_SYNC', None)
  eng = Engine(bench.cfg2_spec())
  eng.init_chains(np.zeros((chains, bench.D)))
  eng.set_rng(rng, seed=7)
  eng.set_collect(moments=moments)
  if trace:
    eng.alloc_trace(steps * (reps + 2), 1)
  eng.run(steps, steps_per_launch=spl)          # warm-up
  walls, enq, kern = [], [], []
  for _ in range(reps):
    eng.sync()
    t0 = time.perf_counter()
    eng.run(steps, steps_per_launch=spl, sync=False)
    t1 = time.perf_counter()
    eng.sync()
    t2 = time.perf_counter()
    walls.append(t2 - t0)
    enq.append(t1 - t0)
    kern.append(eng.last_run_ms()[0] / 1e3)
  eng.close()
  med = lambda v: float(np.median(v))
  out = {'tag': tag, 'rng': rng, 'moments': moments, 'steps': steps, 'chains': chains,
         'sync': sync_env or 'spin',
         'trace': trace, 'spl': spl, 'wall_us': med(walls) * 1e6,
         'enqueue_us': med(enq) * 1e6, 'kernel_us': med(kern) * 1e6,
         'value_wall': chains * steps / med(walls),
         'value_kernel': chains * steps / med(kern),
         'frac_kernel': chains * steps * bench.bytes_per_chain_step(bench.D)
                        / med(kern) / 8e12 if trace else None}
  print(json.dumps(out), flush=True)


if __name__ == '__main__':
  if len(sys.argv) > 1:   # quick form: launch_probe.py TAG STEPS[,STEPS...]
    tag = sys.argv[1]
    for st in [int(v) for v in sys.argv[2].split(',')]:
      out = probe('philox', False, st, 40, None, spl=250, tag=tag)
    sys.exit(0)
  for rng in ('philox', 'philox_fp32'):
    for mom in (False, True):
      probe(rng, mom, 20, 30, None)
  probe('philox', False, 20, 30, 'block')
  probe('philox', False, 250, 8, None)
  probe('philox_fp32', False, 250, 8, None)
  probe('philox', False, 250, 8, None, trace=False)
  probe('philox_fp32', False, 250, 8, None, trace=False)
  probe('xoshiro', False, 250, 8, None)
