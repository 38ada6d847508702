#!/usr/bin/env python3
"""cProfile of SP(samples) -- the summary of a seeded 65 536-chain x 1 000-step
walk (cfg2 shape): where the host time of the trace copy and the PDs goes."""
import cProfile, io, os, pstats, sys
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
for rep in range(2):
  sm = process.sampler(*args, stop=1000, chains=65536, seeds=seeds, steps_per_launch=250, **kwds)
  samples = process.walk(sm)
  pr = cProfile.Profile()
  pr.enable()
  summary = process(samples)
  pr.disable()
  sm.close()
  del summary, samples
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats('tottime').print_stats(25)
print(s.getvalue())
