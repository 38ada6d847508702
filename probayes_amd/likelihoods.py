"""likelihoods.py of the reference (probayes/likelihoods.py) on the GPU path.

bool_perm_freq's row counting runs in the HIP kernel behind the C-ABI entry
pbh_bool_perm_freq (probayes_amd/csrc/pbh_likelihoods.hip).  The small host
parts keep the reference's meaning: the [2] * cols table, the relative
frequencies counts / rows (likelihoods.py:94), and the returned likelihood
function, which slices the table as rf_utils.slice_by_keyvals does
(rf_utils.py:68-164).  int_to_bin / bin_to_int are the reference's host
helpers (likelihoods.py:11-42).
"""
import collections
import ctypes

import numpy as np

from probayes_amd import _lib


def int_to_bin(num, min_dim=0):
  """likelihoods.py:11-26."""
  if isinstance(num, (list, tuple)):
    num = np.array(num, dtype=int)
  if isinstance(num, np.ndarray):
    assert num.ndim == 1, 'Input num must be integer or one dimensional array'
    min_dim = np.maximum(min_dim, len(np.binary_repr(np.max(num))))
    return np.vstack([int_to_bin(element, min_dim) for element in num])
  bits = np.binary_repr(num)
  if min_dim:
    bits = bits.zfill(int(min_dim))
  return np.array([c == '1' for c in bits], dtype=bool)


def bin_to_int(arr, _multiple=None):
  """likelihoods.py:29-42."""
  if isinstance(arr, (list, tuple)):
    arr = np.array(arr, dtype=int)
  assert isinstance(arr, np.ndarray) and arr.ndim and arr.ndim < 3, \
      'Input must be array type of not more than two dimensions'
  if arr.ndim == 2:
    if _multiple is None:
      _multiple = 1 << np.arange(arr.shape[1])[::-1]
    return np.hstack([bin_to_int(row, _multiple) for row in arr])
  if _multiple is None:
    _multiple = 1 << np.arange(arr.size)[::-1]
  return arr.dot(_multiple)


def bool_counts(bool_2d, device=0, reps=1):
  """counts [2] * cols of the row patterns, on the GPU.  Returns (counts,
  average kernel ms)."""
  a = np.ascontiguousarray(bool_2d)
  rows, cols = a.shape
  counts = np.empty(1 << cols, dtype=np.int64)
  ms = ctypes.c_double(0.)
  src = a.view(np.uint8).ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)) \
      if rows else None
  _lib.call('pbh_bool_perm_freq', int(device), int(rows), int(cols), src,
            counts.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), int(reps),
            ctypes.byref(ms))
  return counts.reshape([2] * cols), ms.value


def _isscalar(v):
  return np.isscalar(v) or (isinstance(v, np.ndarray) and v.ndim == 0)


def slice_by_keyvals(spec, vals, prob, vals_dims, spec_dims):
  """rf_utils.py:68-164 for vals_dims / spec_dims given (the only way
  bool_perm_freq's function calls it)."""
  keys = list(spec.keys())
  assert set(keys) == set(vals.keys()), 'Keys for spec and vals unmatched'
  assert set(spec.keys()) == set(spec_dims.keys()), \
      'Keys for spec and spec_dims unmatched'
  vals_ndim = 0
  for dim in vals_dims.values():
    if dim:
      vals_ndim = max(vals_ndim, dim)
  spec_ndim = 0
  for key, dim in spec_dims.items():
    if dim:
      spec_ndim = max(spec_ndim, dim)
    if not _isscalar(spec[key]):
      spec_ndim = max(spec[key].ndim, dim)                   # rf_utils.py:126
  dims = [d for d in vals_dims.values() if d is not None]
  if len(dims) > 1:
    assert np.min(np.diff(dims)) > 0, 'Dimensionality not monotically ordered'
  sdims = [d for d in spec_dims.values() if d is not None]
  if len(sdims) > 1:
    assert np.min(np.diff(sdims)) > 0, 'Dimensionality not monotically ordered'
  reshape = [1] * spec_ndim
  slices = [slice(None) for _ in range(vals_ndim + 1)]
  for key in keys:
    if spec_dims[key] is None:
      dim = vals_dims[key]
      match = np.ravel(vals[key]) == spec[key]
      n_matches = match.sum()
      if n_matches == 0:
        slices[dim] = slice(0, 0)
      elif n_matches == 1:
        slices[dim] = np.nonzero(match)[0]
      else:
        raise ValueError('Non-unique matches found')
    else:
      assert np.all(np.ravel(vals[key]) == np.ravel(spec[key])), \
          'Ambiguous specification with values mismatch'
      reshape[spec_dims[key]] = vals[key].size
  return prob[tuple(slices)].reshape(reshape)


def bool_perm_freq(bool_2d, col_labels=None, base_freq=0, device=0):
  """likelihoods.py:45-101: counts of the boolean permutations in the rows of
  bool_2d, or (likelihood function, relative counts) when labels are given.
  base_freq is accepted and, as in the reference (likelihoods.py:92-94),
  does not change the returned frequencies."""
  assert isinstance(bool_2d, np.ndarray) and bool_2d.ndim == 2 and \
      bool_2d.dtype == bool, 'First input must be a 2D NumPy boolean array'
  rows, cols = bool_2d.shape
  counts, _ = bool_counts(bool_2d, device)
  if col_labels is None:
    return counts
  assert len(col_labels) == cols, \
      'Labels size {} incommensurate with input column number {}'.format(
          len(col_labels), cols)
  dims = collections.OrderedDict()
  vals = collections.OrderedDict()
  ones = np.ones(cols, dtype=int)
  for dim, lbl in enumerate(col_labels):
    reshape = np.copy(ones)
    reshape[dim] = 2
    dims[lbl] = dim
    vals[lbl] = np.array([False, True]).reshape(reshape)
  with np.errstate(invalid='ignore', divide='ignore'):
    rel_freq = counts / rows

  def _func_bool_perm_freq(spec=None, **kwds):
    assert 'dims' in kwds, 'Output dimensionality not given - ' + \
        'use SD.set_prob(function, passdims=True)'
    kwds = dict(kwds)
    spec_dims = kwds.pop('dims')
    if spec is None:
      spec = kwds
    else:
      assert not kwds, 'Unknown keywords: {}'.format(kwds)
    return slice_by_keyvals(spec, vals, rel_freq, dims, spec_dims)

  return _func_bool_perm_freq, rel_freq
