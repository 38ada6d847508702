#!/usr/bin/env python3
"""Reference-identical REPLAY at cfg2 width: the fused kernel (pbh_legacy_run)
against stream generation + the REPLAY kernel, wall time per 250-step launch
(after a warm-up), one JSON line per form.  Usage: replay_fused_probe.py
[chains] [steps] [steps_per_launch]."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from probayes_amd import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
spl = int(sys.argv[3]) if len(sys.argv) > 3 else 250

forms = sys.argv[4].split(',') if len(sys.argv) > 4 else ['fused', 'two_kernel']
for form in forms:
  eng = Engine(bench.cfg2_spec())
  eng.init_chains(np.zeros((n, bench.D)))
  eng.set_rng('replay')
  eng.seed_legacy(np.arange(n))
  eng.alloc_trace(spl + steps, 1)
  eng.reserve_replay(spl)

  def advance(k):
    if form == 'fused':
      eng.legacy_run(k, steps_per_launch=spl, sync=False)
    else:
      for _ in range(k // spl):
        eng.legacy_replay(spl)
        eng.run(spl, sync=False)

  advance(spl)
  eng.sync()
  t0 = time.perf_counter()
  advance(steps)
  eng.sync()
  el = time.perf_counter() - t0
  eng.close()
  print(json.dumps({'form': form, 'pair': os.environ.get('PBH_LEGACY_PAIR', '1'), 'n': n, 'steps': steps, 'spl': spl,
                    'ms_per_launch': el * 1e3 / (steps / spl),
                    'chain_steps_per_s': n * steps / el}), flush=True)
