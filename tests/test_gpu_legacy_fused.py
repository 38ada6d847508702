"""The fused REPLAY kernel (pbh_legacy_run: legacy_mh_kernel generates each
step's draws from the chain's device RandomState straight into the REPLAY
chain-step) against the two-kernel form (pbh_legacy_replay + pbh_run) on
the same seeds: chains, traces (state, log-prob, accept words), moments and
the generator state (the runs that follow) bit-equal, at launch boundaries
of every phase; the forms the fused kernel does not cover (permuted draw
order, per-variable deltas, Gibbs) run as generation + run and equal it too;
the full-width cfg2 run matches the oracle on sampled chains.
"""
import numpy as np
import pytest

import oracle
from oracle.workloads import INITS

pytestmark = pytest.mark.gpu

SIZES = [1, 2, 3, 5, 8, 13, 40]


def _specs():
  out = {name: oracle.golden_spec(name) for name in
         ('diag10', 'gmm2', 'metrohast_norm1d', 'covrw5', 'covrw2', 'mcmc_prob6',
          'bound_sphere2', 'bound_list3', 'fixed2', 'gibbs8')}
  # odd d, identity draw order: the cached polar deviate leads every other step
  s3 = oracle.golden_spec('diag10')
  s3.update(dim=3, names=['x0', 'x1', 'x2'])
  s3['target'] = {'kind': 'diag_gauss', 'mu': np.array([0.5, -1., 0.]),
                  'sigma': np.array([1., 2., 0.5])}
  s3['proposal'] = {'kind': 'gauss', 'loc': np.zeros(3), 'scale': np.full(3, 0.7)}
  s3['ufun'] = np.zeros(3, np.int32)
  out['gauss3'] = s3
  s5 = oracle.golden_spec('diag10')
  s5.update(dim=5, names=['x{}'.format(i) for i in range(5)])
  s5['target'] = {'kind': 'diag_gauss', 'mu': np.zeros(5), 'sigma': np.ones(5)}
  s5['proposal'] = {'kind': 'gauss', 'loc': np.zeros(5), 'scale': np.ones(5),
                    'order': np.array([3, 0, 4, 1, 2], np.int32)}
  s5['ufun'] = np.zeros(5, np.int32)
  out['gauss5_permuted'] = s5
  su = oracle.golden_spec('diag10')
  su['proposal'] = {'kind': 'uniform', 'delta': np.full(10, 0.3)}
  out['uniform10'] = su
  return out


def _init(name, spec, n):
  if name in INITS:
    return np.tile(np.asarray(INITS[name], np.float64), (n, 1))
  return np.zeros((n, int(spec['dim'])))


def _engine(name, spec, n, seeds, cap, thin=1, moments=True):
  from probayes_amd import Engine
  eng = Engine(spec)
  eng.init_chains(_init(name, spec, n))
  eng.set_rng('replay')
  eng.seed_legacy(seeds)
  eng.alloc_trace(cap, thin)
  eng.set_collect(moments)
  return eng


def _state(eng):
  tr = eng.trace()
  out = {k: np.array(tr[k]) for k in ('v_x', 'v_p', 'u') if k in tr}
  x, lp = eng.state()
  out.update({'x': x, 'lp': lp})
  return out


def _equal(a, b, what):
  for k in a:
    assert np.array_equal(a[k], b[k], equal_nan=True), (what, k)


@pytest.mark.parametrize('name', sorted(_specs()))
def test_fused_replay_equals_generation_plus_run(name):
  spec = _specs()[name]
  n = 96                                   # a full and a partial wavefront
  seeds = np.arange(31_000, 31_000 + n)
  total = sum(SIZES) + 7
  two = _engine(name, spec, n, seeds, total)
  one = _engine(name, spec, n, seeds, total)
  for t in SIZES:
    two.legacy_replay(t)
    two.run(t)
    one.legacy_run(t)
    _equal(_state(two), _state(one), (name, t))
  # the generator state: the next steps, both by the two-kernel form
  for eng in (two, one):
    eng.legacy_replay(7)
    eng.run(7)
  _equal(_state(two), _state(one), (name, 'continued'))
  # moments: the lane-pair REPLAY kernel (the two-kernel form at even d >= 4)
  # forms x * x with an fma into sumsq, the one-lane body without
  m2, m1 = two.moments(), one.moments()
  for k in ('sum', 'n_acc', 'n_steps'):
    assert np.array_equal(np.asarray(m2[k]), np.asarray(m1[k])), k
  np.testing.assert_allclose(m1['sumsq'], m2['sumsq'], rtol=1e-14, atol=0)
  two.close()
  one.close()


@pytest.mark.parametrize('name', ['diag10', 'gauss3', 'metrohast_norm1d'])
def test_fused_replay_thin_and_launch_split(name):
  """thin = 3 (records at every phase), steps_per_launch splitting one call,
  and no moments: the same records and state as the two-kernel form."""
  spec = _specs()[name]
  n = 64
  seeds = np.arange(500, 500 + n)
  total = 61
  two = _engine(name, spec, n, seeds, total // 3 + 1, thin=3, moments=False)
  one = _engine(name, spec, n, seeds, total // 3 + 1, thin=3, moments=False)
  two.legacy_replay(total)
  two.run(total, steps_per_launch=9)
  one.legacy_run(total, steps_per_launch=9)
  _equal(_state(two), _state(one), name)
  ms, nl = one.last_run_ms()
  assert nl == 7 and ms > 0.
  two.close()
  one.close()


def test_fused_replay_full_width_cfg2():
  """65 536 chains x 100 steps in 25-step launches: equal to the two-kernel
  form, and to the oracle (NumPy's RandomState streams, the reference's
  arithmetic) on sampled chains."""
  from probayes_amd import Engine
  spec = oracle.golden_spec('diag10')
  n, t = 65536, 100
  seeds = np.arange(n) + 9_000_000
  outs = []
  for fused in (False, True):
    eng = Engine(spec)
    eng.init_chains(np.zeros((n, 10)))
    eng.set_rng('replay')
    eng.seed_legacy(seeds)
    eng.alloc_trace(t, 1)
    if fused:
      eng.legacy_run(t, steps_per_launch=25)
    else:
      for _ in range(4):
        eng.legacy_replay(25)
        eng.run(25)
    outs.append(_state(eng))
    eng.close()
  _equal(outs[0], outs[1], 'cfg2')
  out = outs[1]
  pick = np.random.RandomState(12).choice(n, 128, replace=False)
  ref = oracle.run_mh(spec, np.zeros((128, 10)),
                      oracle.legacy_streams(spec, seeds[pick], t))
  assert np.array_equal(out['u'][pick], ref['u'])
  den = np.maximum(np.abs(ref['v_x']), 1.)
  assert np.max(np.abs(out['v_x'][pick] - ref['v_x']) / den) <= 1e-12


def test_fused_replay_needs_seeded_replay_engine():
  from probayes_amd import Engine
  from probayes_amd._lib import PbhError
  spec = oracle.golden_spec('diag10')
  eng = Engine(spec)
  eng.init_chains(np.zeros((64, 10)))
  eng.set_rng('replay')
  with pytest.raises(PbhError):
    eng.legacy_run(3)                      # not seeded
  eng.seed_legacy(np.arange(64))
  eng.set_rng('philox')
  with pytest.raises(PbhError):
    eng.legacy_run(3)                      # not the REPLAY RNG
  eng.close()
