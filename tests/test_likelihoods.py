"""likelihoods.py (bool_perm_freq, int_to_bin, bin_to_int) against golden
vectors recorded from the reference (tools/gen_likelihood_golden.py).

CPU: the oracle's counting and the host helpers reproduce the golden vectors
exactly.  GPU (-m gpu, through the C-ABI): the HIP histogram reproduces the
golden counts, relative frequencies and likelihood-function outputs exactly,
covers the kernel's three counting paths and ragged tiles, and at 2^28 rows
equals NumPy's bincount (a size-independent check: counts sum to rows).
"""
import json
import os

import numpy as np
import pytest

from likelihood_cases import CASES, make_input, specs_for
from oracle.likelihoods import bool_perm_counts

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden', 'likelihoods.npz')


def _golden():
  with np.load(GOLDEN, allow_pickle=False) as z:
    g = {k: z[k] for k in z.files}
  g['meta'] = json.loads(str(g['meta']))
  return g


def test_golden_inputs_are_the_cases():
  g = _golden()
  assert g['meta']['generator'] == 'tools/gen_likelihood_golden.py'
  for k, case in enumerate(CASES):
    np.testing.assert_array_equal(g['in_{}'.format(k)], make_input(case))


@pytest.mark.parametrize('k', range(len(CASES)))
def test_oracle_counts_match_reference(k):
  g = _golden()
  c = bool_perm_counts(g['in_{}'.format(k)])
  np.testing.assert_array_equal(c, g['counts_{}'.format(k)])
  assert c.dtype == g['counts_{}'.format(k)].dtype


def test_host_helpers_match_reference():
  from probayes_amd.likelihoods import int_to_bin, bin_to_int
  g = _golden()
  np.testing.assert_array_equal(
      np.concatenate([int_to_bin(5), int_to_bin(6, 5)]), g['int_to_bin_scalar'])
  ints = np.array([0, 1, 5, 6, 255, 1023])
  np.testing.assert_array_equal(int_to_bin(ints, 12), g['int_to_bin_vec'])
  np.testing.assert_array_equal(bin_to_int(g['int_to_bin_vec'].astype(int)),
                                g['bin_to_int_vec'])


def test_slice_by_keyvals_matches_reference_on_golden_tables():
  """The host slicing of the returned function, fed the golden rel_freq."""
  from probayes_amd.likelihoods import slice_by_keyvals
  g = _golden()
  for k, case in enumerate(CASES):
    cols = case['cols']
    labels = ['v{}'.format(j) for j in range(cols)]
    vals, dims = {}, {}
    for j, lbl in enumerate(labels):
      shape = [1] * cols
      shape[j] = 2
      vals[lbl] = np.array([False, True]).reshape(shape)
      dims[lbl] = j
    rf = g['rel_freq_{}'.format(k)]
    for i, (spec, sdims) in enumerate(specs_for(cols)):
      out = slice_by_keyvals(spec, vals, rf, dims, sdims)
      np.testing.assert_array_equal(out, g['call_{}_{}'.format(k, i)])


@pytest.mark.gpu
@pytest.mark.parametrize('k', range(len(CASES)))
def test_gpu_bool_perm_freq_matches_reference(k):
  import probayes_amd as pb
  g = _golden()
  a = g['in_{}'.format(k)]
  counts = pb.bool_perm_freq(a)
  np.testing.assert_array_equal(counts, g['counts_{}'.format(k)])
  labels = ['v{}'.format(j) for j in range(a.shape[1])]
  f, rf = pb.bool_perm_freq(a, labels, base_freq=CASES[k].get('base_freq', 0))
  np.testing.assert_array_equal(rf, g['rel_freq_{}'.format(k)])
  for i, (spec, dims) in enumerate(specs_for(a.shape[1])):
    np.testing.assert_array_equal(f(spec, dims=dims),
                                  g['call_{}_{}'.format(k, i)])


@pytest.mark.gpu
@pytest.mark.parametrize('rows,cols', [(1, 1), (17, 1), (3, 2), (1001, 2), (1003, 4),
                                       (255, 4), (256, 4), (257, 5),
                                       (70001, 13), (70001, 14), (4099, 26),
                                       (1 << 20, 7)])
def test_gpu_counts_edge_shapes(rows, cols):
  from probayes_amd.likelihoods import bool_counts
  a = np.random.RandomState(rows + cols).rand(rows, cols) < 0.5
  counts, _ = bool_counts(a)
  np.testing.assert_array_equal(counts, bool_perm_counts(a))


@pytest.mark.gpu
def test_gpu_counts_full_size_vs_bincount():
  from probayes_amd.likelihoods import bool_counts
  rows, cols = 1 << 28, 2
  rs = np.random.RandomState(9)
  a = rs.randint(0, 2, size=(rows, cols), dtype=np.uint8).view(bool)
  counts, ms = bool_counts(a, reps=2)
  assert counts.sum() == rows
  idx = (a[:, 0].astype(np.int64) << 1) | a[:, 1]
  np.testing.assert_array_equal(counts.reshape(-1), np.bincount(idx, minlength=4))
  assert ms > 0


@pytest.mark.gpu
def test_gpu_bool_perm_freq_errors_are_loud():
  from probayes_amd import _lib
  from probayes_amd.likelihoods import bool_counts
  with pytest.raises(AssertionError):
    import probayes_amd as pb
    pb.bool_perm_freq(np.zeros((3, 2), dtype=np.int8))
  with pytest.raises(_lib.PbhError):
    bool_counts(np.zeros((3, 27), bool))
