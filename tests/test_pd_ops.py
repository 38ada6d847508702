"""Summary-PD operations of the facade (probayes_amd/pd.py) against the
reference's PD.expectation / sorted / quantile (pd.py:373-493) on MH
summaries recorded from the reference (tests/golden/pd_ops.npz, made by
tools/gen_pd_golden.py), and the batched [T, N] form chain by chain."""
import json
import os

import numpy as np
import pytest

from probayes_amd.pd import PD

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden',
                    'pd_ops.npz')


def _cases():
  with np.load(GOLD, allow_pickle=False) as z:
    g = {k: z[k] for k in z.files}
  meta = json.loads(str(g['meta']))
  return g, meta


def _pd(g, name, keys):
  return PD('p', {k: g['{}_val_{}'.format(name, k)] for k in keys},
            prob=g['{}_prob'.format(name)], pscale='log')


@pytest.mark.parametrize('case', [0, 1])
def test_summary_ops_match_reference(case):
  g, meta = _cases()
  name, keys = meta['cases'][case]['name'], meta['cases'][case]['keys']
  v = _pd(g, name, keys)
  ex, ex2 = v.expectation(), v.expectation(exponent=2)
  for k in keys:
    assert ex[k] == g['{}_exp_{}'.format(name, k)]
    assert ex2[k] == g['{}_exp2_{}'.format(name, k)]
  srt = v.sorted(keys[0])
  for k in keys:
    np.testing.assert_array_equal(srt[k], g['{}_sorted_{}'.format(name, k)])
  np.testing.assert_array_equal(srt.prob, g['{}_sorted_prob'.format(name)])
  quants = srt.quantile(meta['qs'])
  for k in keys:
    isset = g['{}_quant_isset_{}'.format(name, k)]
    want = g['{}_quant_{}'.format(name, k)]
    for j, qd in enumerate(quants):
      if isset[j]:
        assert qd[k] == {int(want[j])}
      else:
        assert qd[k] == want[j]
  uq = v.quantile(0.5)
  for k, isset in zip(keys, g['{}_unsorted_quant_isset'.format(name)]):
    assert isinstance(uq[k], set) == bool(isset)
  assert v.marginal(keys).keys() == v.keys()
  if len(keys) > 1:
    with pytest.raises(AssertionError):
      v.marginal(keys[0])


def test_batched_summary_ops_are_per_chain():
  g, meta = _cases()
  name, keys = meta['cases'][1]['name'], meta['cases'][1]['keys']
  one = _pd(g, name, keys)
  rev = PD('p', {k: one[k][::-1] for k in keys}, prob=one.prob[::-1],
           pscale='log')
  both = PD('p', {k: np.stack([one[k], rev[k]], 1) for k in keys},
            prob=np.stack([one.prob, rev.prob], 1), pscale='log')
  ex = both.expectation()
  for k in keys:
    np.testing.assert_allclose(ex[k], [one.expectation()[k],
                                       rev.expectation()[k]], rtol=1e-14)
  sb = both.sorted(keys[0])
  s1 = one.sorted(keys[0])
  np.testing.assert_array_equal(sb[keys[0]][:, 0], s1[keys[0]])
  np.testing.assert_array_equal(sb[keys[0]][:, 1], s1[keys[0]])
  qb = sb.quantile([0.25, 0.75])
  q1 = s1.quantile([0.25, 0.75])
  assert qb[0][1][keys[0]] == q1[1][keys[0]]


@pytest.mark.parametrize('case', [0, 1])
def test_conditionalise_raises_as_reference(case):
  """pd.py:214-295 on a summary raises; the exception types were recorded
  from the reference (meta cond_errors: all keys, then the first key)."""
  g, meta = _cases()
  name, keys = meta['cases'][case]['name'], meta['cases'][case]['keys']
  v = _pd(g, name, keys)
  for ks, err in zip([keys, keys[:1]], meta['cases'][case]['cond_errors']):
    with pytest.raises(Exception) as info:
      v.conditionalise(ks)
    assert type(info.value).__name__ == err
  with pytest.raises(AssertionError):
    v.conditionalise('not_a_key')


def test_vectorised_quantile_equals_the_per_chain_restatement():
  """PD.quantile on [T, N] summaries runs vectorised over chains
  (_quantile_batched); every chain's result equals _quantile_1d's (the
  restatement pinned against the reference's recorded quantiles) bit for
  bit: sorted and unsorted keys, ties, flat probabilities, q at 0 and 1,
  log and linear pscales."""
  from probayes_amd.pd import _quantile_1d
  rs = np.random.RandomState(4)
  T, N = 40, 37
  x = np.sort(rs.normal(size=(T, N)), axis=0)
  x[:, 3] = x[::-1, 3]                        # decreasing
  x[:, 5] = rs.normal(size=T)                 # unsorted
  x[10:14, 7] = x[10, 7]                      # ties
  y = rs.normal(size=(T, N))
  cases = [(rs.normal(-3, 2, (T, N)), 'log'),
           (np.log(np.full((T, N), 0.1)), 'log'),
           (rs.uniform(0, 1, (T, N)), 'lin')]
  p2 = cases[2][0]
  p2[:, 9] = 0.
  p2[20, 9] = 1.                              # one non-zero weight
  for prob, ps in cases:
    pd_ = PD('p', {'x': x, 'y': y}, prob=prob, pscale=ps)
    qs = [0., 0.1, 0.25, 0.5, 0.9, 1.]
    got = pd_.quantile(qs)
    for c in range(N):
      ref = _quantile_1d({'x': x[:, c], 'y': y[:, c]}, prob[:, c], ps, qs)
      for a, b in zip(got[c], ref):
        for k in ('x', 'y'):
          if isinstance(b[k], set):
            assert a[k] == b[k]
          else:
            assert a[k] == b[k] or (np.isnan(a[k]) and np.isnan(b[k])), \
                (c, k, a[k], b[k])
    one = pd_.quantile(0.5)
    assert all(isinstance(r, dict) for r in one)
