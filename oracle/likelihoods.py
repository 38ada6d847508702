"""CPU restatement of likelihoods.py:45-101 bool_perm_freq's counting.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  The reference loops over
the rows in Python and increments counts[tuple(sequence)] (likelihoods.py:
67-70); that is a histogram of the rows read as binary numbers with the first
column most significant (C order of a [2] * cols array), which this computes
with np.bincount.  Pinned by tests/golden/likelihoods.npz, recorded from the
reference by tools/gen_likelihood_golden.py.
"""
import numpy as np


def bool_perm_counts(bool_2d):
  a = np.asarray(bool_2d)
  assert a.ndim == 2 and a.dtype == bool
  rows, cols = a.shape
  w = (np.int64(1) << np.arange(cols, dtype=np.int64)[::-1])
  idx = a.astype(np.int64).dot(w) if rows else np.zeros(0, np.int64)
  return np.bincount(idx, minlength=1 << cols).astype(np.int64).reshape(
      [2] * cols)
