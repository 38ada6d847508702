#!/usr/bin/env python3
"""cProfile of the seeded façade sampler's first block (cfg2 shape, 65 536
chains, 1 000 steps): where the host time outside the kernel goes."""
import cProfile, io, os, pstats, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import probayes_amd as pb  # noqa: E402
from mcmc_examples import WORKLOADS  # noqa: E402
builder, params, _, _, _ = WORKLOADS['diag10']
process, init, extra, kwds, keys = builder(pb, params)
args = (init,) if extra is None else (init, extra)
seeds = np.arange(65536) + 12345
def once():
  sm = process.sampler(*args, stop=1000, chains=65536, seeds=seeds, steps_per_launch=250, **kwds)
  next(iter(sm))
  sm.close()
once()
pr = cProfile.Profile()
pr.enable()
once()
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats('cumulative').print_stats(35)
print(s.getvalue())
