"""Cases of the bool_perm_freq golden vectors (tools/gen_likelihood_golden.py)
and the specs the returned likelihood function is called with.  Shared by the
generator (run against the reference) and tests/test_likelihoods.py."""
import numpy as np

CASES = [
    # examples/naive/naive_implicit.py:13-21 (zx_obs shape) and the ballot,
    # LDS-histogram and global-atomic kernel paths (cols <= 4, <= 13, > 13)
    {'rows': 1000, 'cols': 2, 'p': 0.5, 'seed': 1},
    {'rows': 777, 'cols': 1, 'p': 0.3, 'seed': 2},
    {'rows': 5000, 'cols': 5, 'p': 0.4, 'seed': 3, 'base_freq': 1},
    {'rows': 20000, 'cols': 13, 'p': 0.5, 'seed': 4},
    {'rows': 3000, 'cols': 14, 'p': 0.2, 'seed': 5},
    {'rows': 257, 'cols': 3, 'p': 0.7, 'seed': 6},
    {'rows': 0, 'cols': 3, 'p': 0.5, 'seed': 7},
]


def make_input(case):
  rs = np.random.RandomState(case['seed'])
  return rs.rand(case['rows'], case['cols']) < case['p']


def specs_for(cols):
  """(spec, dims) pairs for labels v0..v{cols-1}."""
  labels = ['v{}'.format(j) for j in range(cols)]
  ft = np.array([False, True])
  out = [({k: bool(j % 2) for j, k in enumerate(labels)},
          {k: None for k in labels})]
  if cols <= 6:
    full = {}
    for j, k in enumerate(labels):
      shape = [1] * cols
      shape[j] = 2
      full[k] = ft.reshape(shape)
    out.append((full, {k: j for j, k in enumerate(labels)}))
  if cols >= 2:
    spec = {k: True for k in labels}
    dims = {k: None for k in labels}
    spec[labels[-1]] = ft
    dims[labels[-1]] = 0
    out.append((spec, dims))
  return out
