#!/usr/bin/env python3
"""The driver's bench shape (cfg2, 65 536 chains, 5 one-step warm-up launches,
then 20-step timed launches) in ONE process: per timed launch, the host
enqueue, the wall time to the end of the sync and the HIP-event time, for the
first timed launch and the ones after it.  usage: s20_probe.py TAG"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from probayes_amd import Engine  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else ''
# variants (environment): PROBE_PIN=1 pins the process to its first CPU,
# PROBE_GC=0 disables the garbage collector, PROBE_WARM=k one-step warm-up
# launches (default 5), PROBE_PRIME=1 reads the events once before timing,
# PROBE_WARMLOOP=1 makes each warm-up step its own pbh_run call
if os.environ.get('PROBE_PIN') == '1':
  os.sched_setaffinity(0, {sorted(os.sched_getaffinity(0))[0]})
if os.environ.get('PROBE_GC') == '0':
  import gc
  gc.disable()
warm = int(os.environ.get('PROBE_WARM', '5'))
eng = Engine(bench.cfg2_spec())
eng.init_chains(np.zeros((65536, bench.D)))
eng.set_rng('philox', seed=7)
eng.set_collect(moments=False)
eng.alloc_trace(warm + 20 * 8, 1)
if os.environ.get('PROBE_WARMLOOP') == '1':   # one pbh_run call per step
  for _ in range(warm):
    eng.run(1)
else:
  eng.run(warm, steps_per_launch=1)
eng.sync()
if os.environ.get('PROBE_PRIME') == '1':
  eng.last_run_ms()
rows = []
for i in range(8):
  eng.sync()
  t0 = time.perf_counter()
  eng.run(20, steps_per_launch=250, sync=False)
  t1 = time.perf_counter()
  eng.sync()
  t2 = time.perf_counter()
  ms, _ = eng.last_run_ms()
  rows.append({'tag': tag, 'i': i, 'enqueue_us': (t1 - t0) * 1e6,
               'wall_us': (t2 - t0) * 1e6, 'events_us': ms * 1e3})
eng.close()
for r in rows:
  print(json.dumps(r))
