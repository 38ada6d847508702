"""PD: the result container of the SP facade (mirrors probayes pd.py).

The reference's PD (pd.py:15) is a named dict of variable values plus a
probability `prob` in a given `pscale`; SP.__call__(samples) summates the
per-step PDs into 1-D arrays (pd_utils.py:332-411).  Here the values are the
engine's trace arrays -- [T] for a single chain, [T, N] for a batched sampler
-- and no per-step object is ever built on the hot path.
"""
import numpy as np

from probayes_amd.pscales import rescale


class PD(dict):
  """Named dict of arrays with .prob and .pscale (pd.py:15-45)."""

  def __init__(self, name, values, prob=None, pscale=None):
    super().__init__(values)
    self.name = name
    self.prob = prob
    self.pscale = pscale

  @property
  def keys_list(self):
    return list(self.keys())

  def rescaled(self, pscale=None):
    """pd.py:496-499: prob rescaled from self.pscale to pscale."""
    prob = None if self.prob is None else \
        rescale(np.copy(self.prob), self.pscale, pscale)
    return PD(self.name, dict(self), prob=prob, pscale=pscale)

  def __repr__(self):
    keys = ','.join(self.keys())
    shape = None if self.prob is None else np.shape(self.prob)
    return 'p({})~{}'.format(keys, shape)
