"""Runs the REFERENCE (this container only) on the gibbs_linreg workload with
probayes_amd.linreg.LinRegConditional as the user tfun, and checks that the
reference's chains equal the recorded golden ones (so the descriptor is a
drop-in cond_reg for the reference too).  Recipe as tools/gen_golden.py."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
sys.path.insert(0, ROOT)
import numpy as np

from mcmc_examples import TFUN_WORKLOADS
from probayes_amd.linreg import LinRegConditional
import probayes as pb

builder, params, n, t, seed0 = TFUN_WORKLOADS['gibbs_linreg']
g = np.load(os.path.join(ROOT, 'tests', 'golden', 'gibbs_linreg.npz'))
for c in range(n):
  process, init, extra, kwds, keys = builder(pb, dict(params, cond=LinRegConditional))
  np.random.seed(seed0 + c)
  samples = list(process.walk(process.sampler(init, extra, stop=t, **kwds)))
  vx = np.array([[float(s.v[k]) for k in keys] for s in samples])
  vp = np.array([float(s.v.prob) for s in samples])
  assert np.array_equal(vx, g['v_x'][c]) and np.array_equal(vp, g['v_p'][c]), c
print('reference with LinRegConditional == golden on', n, 'chains x', t, 'steps')
