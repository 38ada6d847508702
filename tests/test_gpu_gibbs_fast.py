"""The production CondCov Gibbs kernel (gibbs_fast_kernel, Philox RNG).

It draws the conditional law of cond_cov.py:42-65 -- the standard normal
truncated to [ndtri(cdf_lo), ndtri(cdf_hi)], scaled and shifted to the
conditional mean / sd -- from fp64 Box-Muller normals (inversion only when a
normal falls outside the limits), and keeps the permuted mvn quadratic form of
v.prob (prob.py:349-358) up to date in O(d) per coordinate.  Checked:
  * v.prob of every recorded step equals scipy's multivariate_normal.pdf at
    the permuted state (1e-9 relative: the O(d) update's rounding drift);
  * posterior moments match the target N(mu, Sigma) within Monte-Carlo error
    for d = 8, 6 (2 lanes per chain), 16 (4 lanes), 3 (1 lane) and 2 with
    tsteps = 2;
  * with tight limits (the inversion fallback is taken often) the moments
    agree with the reference-arithmetic ndtri kernel;
  * traces do not depend on how a run is split into launches or how chains
    are sharded (Philox keyed by global chain id and absolute step).
"""
import numpy as np
import pytest
import scipy.stats

import oracle
from oracle.mh import mvn_perm
from oracle.workloads import _gibbs

pytestmark = pytest.mark.gpu


def _engine(spec, monkeypatch, fast=True):
  from probayes_amd import Engine
  monkeypatch.setenv('PBH_GIBBS_FAST', '1' if fast else '0')
  return Engine(spec)


def _spec_d(d, seed, lo=-20., hi=20.):
  rs = np.random.RandomState(seed)
  a = rs.normal(size=(d, d))
  cov = a @ a.T / d + 0.5 * np.eye(d)
  mean = 0.5 * rs.normal(size=d)
  return _gibbs(mean, cov, lo, hi, ['x{}'.format(i) for i in range(d)])


def _run(spec, monkeypatch, n, t, seed=5, spl=0, n0=0, fast=True, trace=True):
  d = spec['dim']
  eng = _engine(spec, monkeypatch, fast)
  eng.init_chains(np.zeros((n, d)), chain_offset=n0)
  eng.set_rng('philox', seed=seed)
  if trace:
    eng.alloc_trace(t, 1)
  eng.run(t, steps_per_launch=spl)
  out = eng.trace() if trace else None
  mom = eng.moments()
  eng.close()
  return out, mom


@pytest.mark.parametrize('name', ['gibbs8', 'gibbs_norm2d', 'gibbs_sweep2'])
def test_vprob_is_the_permuted_mvn_pdf(name, monkeypatch):
  spec = oracle.golden_spec(name)
  d = spec['dim']
  out, mom = _run(spec, monkeypatch, 300, 600)
  mvn = scipy.stats.multivariate_normal(spec['target']['mean'],
                                        spec['target']['cov'])
  x = out['v_x'].reshape(-1, d)[:, mvn_perm(d)]
  ref = mvn.pdf(x).reshape(out['v_p'].shape)
  np.testing.assert_allclose(out['v_p'], ref, rtol=1e-9, atol=0)
  assert out['u'].all()
  assert np.array_equal(mom['n_acc'], np.full(300, 600))
  np.testing.assert_allclose(mom['sum'], out['v_x'].sum(axis=1), rtol=1e-12,
                             atol=1e-9)


@pytest.mark.parametrize('case', ['gibbs8', 'd6', 'd3', 'd16', 'gibbs_sweep2'])
def test_posterior_moments_match_target(case, monkeypatch):
  spec = (oracle.golden_spec(case) if case.startswith('gibbs')
          else _spec_d(int(case[1:]), 7))
  d = spec['dim']
  n, burn, t = 8192, 10 * d, 200 * d
  from probayes_amd import Engine
  monkeypatch.setenv('PBH_GIBBS_FAST', '1')
  eng = Engine(spec)
  eng.init_chains(np.zeros((n, d)))
  eng.set_rng('philox', seed=21)
  eng.run(burn)
  eng.reset_moments()
  eng.run(t - burn)
  mom = eng.moments()
  eng.close()
  steps = mom['n_steps']
  mean = mom['sum'].sum(0) / (n * steps)
  var = mom['sumsq'].sum(0) / (n * steps) - mean ** 2
  mu = np.asarray(spec['target']['mean'])
  sd = np.sqrt(np.diag(spec['target']['cov']))
  assert np.all(np.abs(mean - mu) < 0.03 * sd), (mean, mu)
  assert np.all(np.abs(var / sd ** 2 - 1) < 0.03), var / sd ** 2


def test_tight_limits_match_the_ndtri_kernel(monkeypatch):
  """Limits at about one sd: the inversion fallback runs on a large share of
  draws; the law must equal the reference-arithmetic kernel's."""
  spec = _gibbs([0.5, -0.5], [[1.5, -1.0], [-1.0, 2.]], -0.5, 1.0,
                ['x', 'y'])
  n, t = 16384, 400
  res = []
  for fast in (True, False):
    out, _ = _run(spec, monkeypatch, n, t, seed=3, fast=fast)
    v = out['v_x'][:, 40:].reshape(-1, 2)
    res.append((v.mean(0), v.var(0), np.corrcoef(v.T)[0, 1]))
  (m1, v1, c1), (m0, v0, c0) = res
  np.testing.assert_allclose(m1, m0, atol=0.01)
  np.testing.assert_allclose(v1, v0, rtol=0.02)
  assert abs(c1 - c0) < 0.01


def test_launch_split_and_sharding_invariance(monkeypatch):
  spec = oracle.golden_spec('gibbs8')
  full, _ = _run(spec, monkeypatch, 4096, 300, seed=9)
  split, _ = _run(spec, monkeypatch, 4096, 300, seed=9, spl=37)
  lo, _ = _run(spec, monkeypatch, 1000, 300, seed=9)
  hi, _ = _run(spec, monkeypatch, 3096, 300, seed=9, n0=1000)
  for k in ('v_x', 'v_p', 'u'):
    np.testing.assert_array_equal(full[k], split[k])
    np.testing.assert_array_equal(full[k][:1000], lo[k])
    np.testing.assert_array_equal(full[k][1000:], hi[k])
