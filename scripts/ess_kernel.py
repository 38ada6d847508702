#!/usr/bin/env python3
"""The device ESS of cfg5's trace alone (for PMC passes): 32 768 chains of
gmm2, 2 000 steps recorded, then pbh_trace_ess over records [500, 2000)
(2 x 32 768 series of 1 500), twice (a warm-up and the measured call)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
from oracle.workloads import golden_init  # noqa: E402
from probayes_amd import Engine  # noqa: E402

eng = Engine(oracle.golden_spec('gmm2'))
eng.init_chains(golden_init('gmm2', 32768))
eng.set_rng('philox', seed=11)
eng.set_collect(moments=False)
eng.alloc_trace(2000, 1)
eng.run(2000, steps_per_launch=250)
eng.sync()
ess = eng.trace_ess(500)
t0 = time.perf_counter()
ess = eng.trace_ess(500)
print('ess call ms', (time.perf_counter() - t0) * 1e3, 'min', float(ess.min()), 'mean', float(ess.mean()))
eng.close()
