#!/usr/bin/env python3
"""Where a seeded sampler's first block spends its time: the engine calls the
façade makes (Sampler._start_epoch / _compute_engine), each timed."""
import json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from probayes_amd import Engine  # noqa: E402
n, T = 65536, 1000
for rep in range(3):
  tt = {}
  def lap(k, t0=[time.perf_counter()]):
    t = time.perf_counter(); tt[k] = round((t - t0[0]) * 1e3, 3); t0[0] = t
  lap('start')
  eng = Engine(bench.cfg2_spec()); lap('create')
  eng.init_chains(np.zeros((n, 10))); lap('init_chains')
  eng.set_rng('replay'); lap('set_rng')
  eng.seed_legacy(np.arange(n) + 1); lap('seed_legacy')
  eng.set_record_threshold(True); lap('record_thr')
  eng.state(); lap('state')
  eng.alloc_trace(T, 1); lap('alloc_trace')
  eng.legacy_run(T, steps_per_launch=250); lap('legacy_run')
  eng.sync(); lap('sync')
  eng.close(); lap('close')
  print(json.dumps(tt), flush=True)
