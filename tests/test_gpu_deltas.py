"""Delta forms beyond the callable / plain tuple / plain list (SURVEY.md §8
a3) in the production modes: bound=True clamps and bounces
(variable.py:700-739), per-variable polarity / uniform / fixed / randint
deltas (variable.py:600-640), int variables (revtype truncation).

Replay parity with the reference's recorded chains runs in
test_gpu_parity.py::test_replay_matches_reference_golden and in
test_facade.py (these workloads are in oracle.WORKLOADS / DELTA_WORKLOADS).
Here the Philox chains are checked against the oracle's chains on NumPy
streams -- the reference's law -- by two-sample tests on the state
distribution at fixed steps (clamped proposals are not symmetric, so the
target alone is not the reference), and by the invariants every proposal
satisfies."""
import numpy as np
import pytest

import oracle
from oracle.workloads import golden_init

pytestmark = pytest.mark.gpu

NAMES = ['bound_sphere2', 'bound_list3', 'pervar3', 'randint2', 'fixed2']


def _philox(spec, init, t, seed, debug=False, mode='philox'):
  from probayes_amd import Engine
  eng = Engine(spec)
  eng.init_chains(init)
  eng.set_rng(mode, seed=seed)
  eng.alloc_trace(t, 1, debug=debug)
  eng.run(t, steps_per_launch=37)
  tr = eng.trace()
  eng.close()
  return tr


@pytest.mark.parametrize('name', NAMES)
@pytest.mark.parametrize('mode', ['philox', 'philox_f64'])
def test_production_law_matches_oracle(name, mode):
  spec = oracle.golden_spec(name)
  n_gpu, n_cpu, t = 32768, 4096, 96
  g = _philox(spec, golden_init(name, n_gpu), t, seed=5, mode=mode)
  r = oracle.run_mh(spec, golden_init(name, n_cpu),
                    oracle.legacy_streams(spec, np.arange(900, 900 + n_cpu), t))
  for step in (7, t - 1):
    a, b = g['v_x'][:, step], r['v_x'][:, step]
    for k in range(a.shape[1]):
      sa, sb = a[:, k].std(), b[:, k].std()
      se = np.sqrt(sa ** 2 / n_gpu + sb ** 2 / n_cpu)
      if se == 0:          # a degenerate coordinate (e.g. clamped at a limit)
        assert np.array_equal(np.unique(a[:, k]), np.unique(b[:, k]))
        continue
      assert abs(a[:, k].mean() - b[:, k].mean()) <= 5 * se, (step, k)
      # variances, with the sampling error of s^2 from the fourth moment
      # (the state laws are skewed and discrete near fixed steps / limits)
      va, vb = sa ** 2, sb ** 2
      m4a = np.mean((a[:, k] - a[:, k].mean()) ** 4)
      m4b = np.mean((b[:, k] - b[:, k].mean()) ** 4)
      se_v = np.sqrt((m4a - va ** 2) / n_gpu + (m4b - vb ** 2) / n_cpu)
      assert abs(va - vb) <= 5 * se_v + 1e-12 * vb, (step, k, va, vb)
  pa, pb = g['u'].mean(), r['u'].mean()
  assert abs(pa - pb) <= 5 * np.sqrt(pb * (1 - pb) / (n_cpu * t)) + 1e-3


@pytest.mark.parametrize('name', NAMES)
def test_proposals_respect_bounds_and_integrality(name):
  spec = oracle.golden_spec(name)
  n, t = 4096, 64
  tr = _philox(spec, golden_init(name, n), t, seed=17, debug=True)
  prop = spec['proposal']
  px, vx = tr['p_x'], tr['v_x']
  b = prop.get('bound')
  for k in range(int(spec['dim'])):
    if b is not None and b['on'][k]:
      lo, hi = b['lo'][k], b['hi'][k]
      # clamped or bounced: never outside the closed limits
      assert px[:, :, k].min() >= lo and px[:, :, k].max() <= hi, k
      if b['xlo'][k] and b['xhi'][k]:
        inside = (px[:, :, k] > lo) & (px[:, :, k] < hi)
        assert inside.all()
    if prop.get('vint') is not None and prop['vint'][k]:
      assert np.array_equal(px[:, :, k], np.trunc(px[:, :, k]))
      assert np.array_equal(vx[:, :, k], np.trunc(vx[:, :, k]))
  if prop['kind'] == 'vardelta':
    # one step's delta per mode: fixed steps exact, polarity +-d
    x0 = golden_init(name, n)
    dl = px[:, 0] - x0
    for k, (m, d0) in enumerate(zip(prop['mode'], prop['delta'])):
      sel = np.ones(n, bool)
      if b is not None and b['on'][k]:   # away from the limits
        sel = (px[:, 0, k] > b['lo'][k]) & (px[:, 0, k] < b['hi'][k])
      if m == 0:
        np.testing.assert_allclose(dl[sel, k], d0, rtol=0, atol=1e-15)
      elif m == 1:
        assert set(np.round(np.abs(dl[sel, k]), 12)) == {round(d0, 12)}
        assert 0.45 < np.mean(dl[sel, k] > 0) < 0.55
      elif m == 3:
        vals = np.unique(dl[sel, k])
        assert set(vals) <= set(range(-int(d0), int(d0)))


def test_randint_values_are_uniform():
  """randint(-3, 3) from Philox words: the six values equally likely."""
  spec = oracle.golden_spec('randint2')
  spec = dict(spec, proposal=dict(spec['proposal'], bound=None))
  n, t = 65536, 4
  init = np.tile([1000., 0.], (n, 1))      # far from any limit
  tr = _philox(spec, init, t, seed=3, debug=True)
  dl = tr['p_x'][:, 0, 0] - 1000.
  counts = np.array([np.sum(dl == v) for v in range(-3, 3)])
  assert counts.sum() == n
  e = n / 6
  assert np.all(np.abs(counts - e) <= 5 * np.sqrt(e)), counts
