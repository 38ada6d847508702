"""Summary operations on ENGINE traces: the device
reductions (pbh_trace_expectation, pbh_trace_stats) against the facade's PD
ops applied to the same trace copied to the host, and the vectorised PD
quantile / sorted / expectation of a batched summary against the per-chain
restatement."""
import numpy as np
import pytest

import oracle
from oracle.workloads import golden_init
from probayes_amd.pd import PD, _quantile_1d

pytestmark = pytest.mark.gpu


def _run(name, n, t, seed=3):
  from probayes_amd import Engine
  spec = oracle.golden_spec(name)
  eng = Engine(spec)
  eng.init_chains(golden_init(name, n))
  eng.set_rng('philox', seed=seed)
  eng.alloc_trace(t, 1)
  eng.run(t, steps_per_launch=64)
  return spec, eng


@pytest.mark.parametrize('name', ['diag10', 'gmm2', 'mcmc_prob4a'])
def test_device_expectation_and_moments_equal_the_pd_ops(name):
  n, t, first = 2000 + 3, 160, 40
  spec, eng = _run(name, n, t)
  try:
    tr = eng.trace()
    keys = spec['names']
    vals = {k: tr['v_x'][:, first:, i].T for i, k in enumerate(keys)}   # [T, N]
    pd_ = PD('v', vals, prob=tr['v_p'][:, first:].T, pscale=spec['pscale'])
    for ex in (None, 2., 3.):
      dev = eng.trace_expectation(first, t - first, exponent=ex)     # [N, d]
      host = pd_.expectation(exponent=ex)
      for i, k in enumerate(keys):
        a, b = dev[:, i], host[k]
        ok = np.isfinite(b)
        assert np.array_equal(np.isfinite(a), ok)
        # relative to the summands' scale max|v|^e: a probability-weighted
        # mean near 0 (a coordinate of a centred target) carries the
        # summation order's rounding of terms ~|v|^e
        scale = np.abs(vals[k]).max(axis=0)[ok] ** (1. if ex is None else ex)
        rel = np.abs(a[ok] - b[ok]) / np.maximum(np.maximum(np.abs(b[ok]), scale), 1e-300)
        assert rel.max() <= 1e-12, (ex, k, rel.max())
    st = eng.trace_stats(first, t - first)
    np.testing.assert_allclose(st['sum'], tr['v_x'][:, first:].sum(1),
                               rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(st['sumsq'], (tr['v_x'][:, first:] ** 2).sum(1),
                               rtol=1e-12, atol=1e-12)
    assert np.array_equal(st['n_acc'], tr['u'][:, first:].sum(1))
  finally:
    eng.close()


def test_batched_quantile_on_engine_trace():
  """Sorted summaries of 4099 engine chains: the vectorised quantile equals
  the per-chain restatement for every chain."""
  spec, eng = _run('diag10', 4096 + 3, 80)
  try:
    tr = eng.trace()
  finally:
    eng.close()
  vals = {k: tr['v_x'][:, :, i].T for i, k in enumerate(spec['names'][:2])}
  pd_ = PD('v', vals, prob=tr['v_p'].T, pscale='log').sorted('x0')
  qs = [0.05, 0.5, 0.95]
  got = pd_.quantile(qs)
  for c in range(0, 4099, 97):
    ref = _quantile_1d({k: v[:, c] for k, v in pd_.items()}, pd_.prob[:, c],
                       'log', qs)
    for a, b in zip(got[c], ref):
      for k in vals:
        assert (a[k] == b[k]) if isinstance(b[k], set) else \
            (a[k] == b[k] or (np.isnan(a[k]) and np.isnan(b[k])))
