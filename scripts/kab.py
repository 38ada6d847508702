#!/usr/bin/env python3
"""Kernel-level A/B of engine knobs (environment read at pbh_create) at the
driver's shape: one engine per configuration in ONE process, 20-step FULL
launches interleaved across the configurations, per-launch HIP-event time
and wall time; prints the medians.
usage: kab.py TAG REPS STEPS "name:VAR=v,VAR=v" ...   (STEPS per launch)"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from probayes_amd import Engine  # noqa: E402

tag, reps, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
cfgs = []
for arg in sys.argv[4:]:
  name, _, envs = arg.partition(':')
  env = dict(kv.split('=', 1) for kv in envs.split(',') if kv)
  saved = {k: os.environ.get(k) for k in env}
  os.environ.update(env)
  eng = Engine(bench.cfg2_spec())
  for k, v in saved.items():
    if v is None:
      os.environ.pop(k)
    else:
      os.environ[k] = v
  eng.init_chains(np.zeros((65536, bench.D)))
  eng.set_rng('philox', seed=7)
  eng.set_collect(moments=False)
  eng.alloc_trace(5 + steps * (reps + 2), 1)
  for _ in range(5):
    eng.run(1)
  eng.run(steps, steps_per_launch=steps)   # untimed
  eng.sync()
  cfgs.append((name, eng, []))
for r in range(reps):
  for name, eng, out in cfgs:
    eng.sync()
    t0 = time.perf_counter()
    eng.run(steps, steps_per_launch=steps, sync=False)
    t1 = time.perf_counter()
    eng.sync()
    t2 = time.perf_counter()
    ms, _ = eng.last_run_ms()
    out.append((ms * 1e3, (t2 - t0) * 1e6, (t1 - t0) * 1e6))
for name, eng, out in cfgs:
  a = np.array(out)
  print(json.dumps({'tag': tag, 'cfg': name, 'steps': steps, 'reps': reps,
                    'events_med': float(np.median(a[:, 0])),
                    'events_p10': float(np.percentile(a[:, 0], 10)),
                    'events_p90': float(np.percentile(a[:, 0], 90)),
                    'wall_med': float(np.median(a[:, 1])),
                    'enq_med': float(np.median(a[:, 2]))}), flush=True)
  eng.close()
