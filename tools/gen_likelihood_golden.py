"""Golden vectors for likelihoods.py (bool_perm_freq, int_to_bin, bin_to_int),
recorded by running the REFERENCE probayes in the build container only.

Recipe:
    PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg PYTHONPATH=/tmp/stub:/root/reference \
        python3 tools/gen_likelihood_golden.py
Writes tests/golden/likelihoods.npz: per case k the input bool array
in_k [rows, cols], counts_k, rel_freq_k (labels given) and, for the labelled
cases, the outputs of the returned function for a fixed list of specs
(scalar and [False, True] values, dims None / 0 / 1 ...; the spec list is
rebuilt by tests/test_likelihoods.py from the same seeds).
"""
import json
import os
import sys

import numpy as np

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   'tests', 'golden', 'likelihoods.npz')
sys.path.insert(0, os.path.join(os.path.dirname(OUT), '..'))
from likelihood_cases import CASES, make_input, specs_for  # noqa: E402


def main():
  import probayes as pb
  from probayes import likelihoods as lk
  out = {}
  meta = {'cases': [], 'numpy': np.__version__,
          'reference': 'probayes 0.0.8 (/root/reference)',
          'generator': 'tools/gen_likelihood_golden.py'}
  for k, case in enumerate(CASES):
    a = make_input(case)
    out['in_{}'.format(k)] = a
    out['counts_{}'.format(k)] = pb.bool_perm_freq(a)
    labels = ['v{}'.format(j) for j in range(a.shape[1])]
    with np.errstate(invalid='ignore', divide='ignore'):
      f, rf = pb.bool_perm_freq(a, labels, base_freq=case.get('base_freq', 0))
    out['rel_freq_{}'.format(k)] = rf
    for i, (spec, dims) in enumerate(specs_for(a.shape[1])):
      out['call_{}_{}'.format(k, i)] = np.asarray(f(spec, dims=dims))
    meta['cases'].append(case)
  ints = np.array([0, 1, 5, 6, 255, 1023])
  out['int_to_bin_scalar'] = np.concatenate([lk.int_to_bin(5),
                                             lk.int_to_bin(6, 5)])
  out['int_to_bin_vec'] = lk.int_to_bin(ints, 12)
  out['bin_to_int_vec'] = lk.bin_to_int(out['int_to_bin_vec'].astype(int))
  out['meta'] = np.array(json.dumps(meta))
  np.savez_compressed(OUT, **out)
  print('wrote', OUT, len(CASES), 'cases')


if __name__ == '__main__':
  main()
