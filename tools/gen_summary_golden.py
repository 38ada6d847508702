"""Golden vectors for the SP summary's o / q / r fields (sp.py:131-198):
runs the REFERENCE (this container only, never on the GPU box) for a few
example workloads, one chain each, and records every field of
`process(samples)` that is a PD: its keys in order, the values of the
variable keys (data keys such as the iid `x` are recorded as skipped) and
its prob.

Recipe: as tools/gen_golden.py (h5py stub, PYTHONPATH=/root/reference).
Output: tests/golden/summary_oqr.npz
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tests'))

from mcmc_examples import WORKLOADS  # noqa: E402

NAMES = ['mcmc_prob6', 'diag10', 'metrohast_norm1d', 'mcmc_prob2']
STEPS = 12


def main():
  import probayes as pb
  import probayes.prob as P
  P.SCIPY_DIST_METHODS = [m for m in P.SCIPY_DIST_METHODS if m != 'fit']
  out, meta = {}, {}
  for name in NAMES:
    builder, params, n, t, seed0 = WORKLOADS[name]
    process, init, extra, kwds, keys = builder(pb, params)
    np.random.seed(seed0)
    args = (init,) if extra is None else (init, extra)
    samples = list(process.walk(process.sampler(*args, stop=STEPS, **kwds)))
    s = process(samples)
    meta[name] = {'seed': seed0, 'steps': STEPS, 'fields': {}}
    for f in ('o', 'p', 'q', 'r'):
      d = getattr(s, f)
      if d is None:
        meta[name]['fields'][f] = None
        continue
      fkeys = [k for k in d.keys() if k.rstrip("'") in keys]
      meta[name]['fields'][f] = fkeys
      for k in fkeys:
        out['{}/{}/{}'.format(name, f, k)] = np.asarray(np.ravel(d[k]), np.float64)
      out['{}/{}/prob'.format(name, f)] = np.asarray(np.ravel(d.prob), np.float64)
  out['meta'] = np.array(json.dumps(meta))
  np.savez_compressed(os.path.join(ROOT, 'tests', 'golden', 'summary_oqr.npz'), **out)
  print(json.dumps(meta, indent=1))


if __name__ == '__main__':
  main()
