"""PD: the result container of the SP facade (mirrors probayes pd.py).

The reference's PD (pd.py:15) is a named dict of variable values plus a
probability `prob` in a given `pscale`; SP.__call__(samples) summates the
per-step PDs into 1-D arrays (pd_utils.py:332-411).  Here the values are the
engine's trace arrays -- [T] for a single chain, [T, N] for a batched sampler
-- and no per-step object is ever built on the hot path.

Summary operations: expectation, sorted, quantile and
marginal with the reference's semantics (pd.py:168-211, 373-493) on the
sample axis -- axis 0, so a batched [T, N] summary is treated chain by
chain.  Pinned by tests/golden/pd_ops.npz (tools/gen_pd_golden.py).
"""
import numpy as np

from probayes_amd.pscales import NEARLY_POSITIVE_ZERO, rescale


def _div_prob(dividend, divisor):
  """pscales.py:219-236 on linear arrays."""
  return dividend / np.maximum(NEARLY_POSITIVE_ZERO, divisor)


def _ismonotonic(vals):
  """pd_utils.py:414-421."""
  vals = np.ravel(vals)
  if vals.size <= 1:
    return True
  return len(np.unique(vals[1:] >= vals[:-1])) == 1


def _quantile_1d(vals, prob, pscale, quants):
  """pd.py:408-460 for one chain's samples (1-D values of every key)."""
  unsorted = {k for k, v in vals.items() if not _ismonotonic(v)}
  ravprob = rescale(np.ravel(np.asarray(prob, float)), pscale, 'lin')
  cumprob = np.cumsum(ravprob)
  cumprob = _div_prob(cumprob, cumprob[-1])
  cum_idx = np.maximum(0, np.digitize(np.array(quants), cumprob) - 1).tolist()
  out = []
  for j, rav_idx in enumerate(cum_idx):
    rav_idx = int(rav_idx)
    qd = {}
    for key, v in vals.items():
      v = np.ravel(v)
      if key in unsorted:
        qd[key] = {v.size}
        continue
      idx = min(rav_idx, len(v) - 1)
      if idx == len(v) - 1:
        qd[key] = v[idx]
        continue
      vv = v[idx:idx + 2]
      ravp = ravprob[rav_idx:rav_idx + 2]
      if np.abs(np.diff(ravp)) < min(quants[j], 1. - quants[j]):
        qd[key] = np.interp(quants[j], cumprob[rav_idx:rav_idx + 2], vv)
      else:
        qd[key] = np.sum(ravp * vv) / np.sum(ravp)
    out.append(qd)
  return out


def _interp2(x, c0, c1, v0, v1):
  """np.interp(x, [c0, c1], [v0, v1]) elementwise, NumPy's own arithmetic
  (numpy/_core/src/multiarray/compiled_base.c arr_interp): below -> v0,
  above or at c1 -> v1, at c0 -> v0, else slope (x - c0) + v0 with the
  NaN fallbacks."""
  with np.errstate(divide='ignore', invalid='ignore'):
    slope = (v1 - v0) / (c1 - c0)
    mid = slope * (x - c0) + v0
    alt = slope * (x - c1) + v1
    mid = np.where(np.isnan(mid), np.where(np.isnan(alt) & (v0 == v1), v0, alt),
                   mid)
  out = np.where(x == c0, v0, mid)
  out = np.where(x >= c1, v1, out)
  return np.where(x < c0, v0, out)


def _quantile_batched(vals, prob, pscale, quants):
  """_quantile_1d for every chain of [T, N] summaries at once (the same
  operations, vectorised over the chain axis): one dict per quantile per
  chain, as the per-chain loop returns."""
  prob = np.asarray(prob, float)
  T, N = prob.shape
  ravprob = rescale(prob, pscale, 'lin')
  cumprob = np.cumsum(ravprob, axis=0)
  cumprob = _div_prob(cumprob, cumprob[-1])
  cols = np.arange(N)
  per_q = []
  for q in quants:
    # np.digitize(q, cumprob) on non-decreasing bins = #{bins <= q}
    ridx = np.maximum(0, np.sum(cumprob <= q, axis=0) - 1)
    res = {}
    for key, v in vals.items():
      v = np.asarray(v).reshape(T, N)
      if T > 1:
        d = v[1:] >= v[:-1]
        mono = d.all(axis=0) | (~d).all(axis=0)
      else:
        mono = np.ones(N, bool)
      idx = np.minimum(ridx, T - 1)
      last = idx == T - 1
      i1 = np.minimum(idx + 1, T - 1)
      v0, v1 = v[idx, cols], v[i1, cols]
      p0, p1 = ravprob[idx, cols], ravprob[i1, cols]
      c0, c1 = cumprob[idx, cols], cumprob[i1, cols]
      near = np.abs(p1 - p0) < min(q, 1. - q)
      with np.errstate(divide='ignore', invalid='ignore'):
        weighted = (p0 * v0 + p1 * v1) / (p0 + p1)
      got = np.where(last, v0, np.where(near, _interp2(q, c0, c1, v0, v1),
                                        weighted))
      res[key] = (got, mono)
    per_q.append(res)
  out = []
  for c in range(N):
    chain = []
    for res in per_q:
      chain.append({k: (g[c] if m[c] else {T}) for k, (g, m) in res.items()})
    out.append(chain)
  return out


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

  def _lin_prob(self):
    return rescale(np.asarray(self.prob, float), self.pscale, 'lin')

  def expectation(self, keys=None, exponent=None):
    """pd.py:373-405: probability-weighted mean over the sample axis,
    sum(p v^exponent) / sum(p) with p rescaled to linear."""
    keys = list(self.keys()) if keys is None else \
        ([keys] if isinstance(keys, str) else list(keys))
    for key in keys:
      assert key in self, 'Key {} not marginal in distribution {}'.format(
          key, self.name)
    prob = self._lin_prob()
    sum_prob = np.sum(prob, axis=0)
    out = {}
    for key in keys:
      val = np.asarray(self[key], float)
      val = val ** exponent if exponent else val
      out[key] = _div_prob(np.sum(prob * val, axis=0), sum_prob)
    return out

  def sorted(self, key):
    """pd.py:463-493: samples reordered by the values of key (argsort along
    the sample axis, per chain when batched)."""
    idx = np.argsort(np.asarray(self[key]), axis=0)
    take = lambda a: np.take_along_axis(np.asarray(a), idx, axis=0)
    vals = {k: take(v) for k, v in self.items()}
    return PD(self.name, vals, prob=take(self.prob), pscale=self.pscale)

  def quantile(self, q=0.5):
    """pd.py:408-460: quantiles of the probability-weighted samples, for
    keys whose values are sorted (others give {size}); batched summaries
    return one dict per chain."""
    scalar = np.isscalar(q)
    quants = [q] if scalar else list(q)
    prob = np.asarray(self.prob, float)
    if prob.ndim <= 1:
      res = _quantile_1d(dict(self), prob, self.pscale, quants)
      return res[0] if scalar else res
    res = _quantile_batched(dict(self), prob, self.pscale, quants)
    return [r[0] if scalar else r for r in res]

  def marginal(self, keys):
    """pd.py:168-211 for a summary, whose variables share the sample axis:
    only the marginal of all of them exists."""
    keys = {keys} if isinstance(keys, str) else set(keys)
    for key in keys:
      assert key in self, 'Key {} not marginal in distribution {}'.format(
          key, self.name)
    assert keys == set(self.keys()), \
        'Dimensionality precludes marginalising {} without: {}'.format(
            keys, set(self.keys()) - keys)
    return PD(self.name, dict(self), prob=self.prob, pscale=self.pscale)

  def conditionalise(self, keys):
    """pd.py:214-295.  On an MH / Gibbs summary every variable shares the
    sample axis (dims {key: 0}); the reference then fails inside its own
    arithmetic: conditionalising all keys sums over ``axis=None * ...`` and
    raises TypeError, a strict subset moves axis 0 to axis 1 of a 1-D prob and
    raises numpy's AxisError (recorded from the reference in
    tests/golden/pd_ops.npz, ``cond_errors``).  The summary raises the same
    exception types, so ``SP(samples, conditionalise=True)`` (sp.py:132-149,
    196-197) fails as it does in the reference."""
    keys = {keys} if isinstance(keys, str) else set(keys)
    for key in keys:
      assert key in self, 'Key {} not marginal in distribution {}'.format(
          key, self.name)
    if keys == set(self.keys()):
      raise TypeError("unsupported operand type(s) for *: 'NoneType' and "
                      "'int' (pd.py:284: summary prob has no axis to "
                      "normalise over)")
    raise np.exceptions.AxisError(1, 1, 'destination')

  def __repr__(self):
    keys = ','.join(self.keys())
    shape = None if self.prob is None else np.shape(self.prob)
    return 'p({})~{}'.format(keys, shape)
