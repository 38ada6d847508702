"""Device-generated reference streams (pbh_legacy_seed / pbh_legacy_replay):
one NumPy legacy RandomState per chain (MT19937 init_genrand seeding,
random_sample, polar legacy gauss with its cached deviate) drawn on the GPU in
the reference's per-step order, against NumPy's own
RandomState (oracle.legacy_streams):
  * uniform draws (random_sample) bit-identical;
  * normal draws identical up to the device log's last-ulp rounding
    (<= 4e-16 relative; the polar method's log(r2) is the only libm call);
  * generator state persists across calls (MT position, cached gauss);
  * a full-width cfg2 replay run fed by device streams matches the oracle
    on sampled chains step for step.
"""
import numpy as np
import pytest

import oracle
from oracle.workloads import golden_init

pytestmark = pytest.mark.gpu


def _engine(spec, n, seeds):
  from probayes_amd import Engine
  eng = Engine(spec)
  eng.init_chains(golden_init_like(spec, n))
  eng.seed_legacy(seeds)
  return eng


def golden_init_like(spec, n):
  return np.zeros((n, int(spec['dim'])))


def _specs():
  out = {name: oracle.golden_spec(name) for name in
         ('diag10', 'gmm2', 'metrohast_norm1d', 'covrw5', 'gibbs8',
          'gibbs_sweep2', 'mcmc_prob6')}
  # odd d with the Gaussian delta: the cached polar deviate crosses steps
  s5 = oracle.golden_spec('diag10')
  s5.update(dim=5, names=['x{}'.format(i) for i in range(5)])
  s5['target'] = {'kind': 'diag_gauss', 'mu': np.zeros(5), 'sigma': np.ones(5)}
  s5['proposal'] = {'kind': 'gauss', 'loc': np.zeros(5), 'scale': np.ones(5),
                    'order': np.array([3, 0, 4, 1, 2], np.int32)}
  s5['ufun'] = np.zeros(5, np.int32)
  out['gauss5_permuted'] = s5
  # list (uniform) delta
  su = oracle.golden_spec('diag10')
  su['proposal'] = {'kind': 'uniform', 'delta': np.full(10, 0.3)}
  out['uniform10'] = su
  # per-variable deltas: randint (NumPy's masked rejection on 32-bit words,
  # small and wide ranges, a float bound truncated), polarity, fixed
  for name in ('randint2', 'pervar3'):
    out[name] = oracle.golden_spec(name)
  sv = oracle.golden_spec('diag10')
  sv.update(dim=4, names=['a', 'b', 'c', 'e'])
  sv['target'] = {'kind': 'diag_gauss', 'mu': np.zeros(4), 'sigma': np.ones(4)}
  sv['proposal'] = {'kind': 'vardelta', 'mode': np.array([3, 3, 1, 0], np.int32),
                    'delta': np.array([1000., 70000.5, 0.3, 0.2]),
                    'vint': np.array([1, 1, 0, 0], np.int32)}
  sv['ufun'] = np.zeros(4, np.int32)
  out['randint_wide'] = sv
  return out


def _check(dev, ref, normal_rows):
  both_nan = np.isnan(dev) & np.isnan(ref)
  assert np.array_equal(np.isnan(dev), np.isnan(ref))
  dev, ref = np.where(both_nan, 0., dev), np.where(both_nan, 0., ref)
  for j in range(ref.shape[1]):
    if j in normal_rows:
      rel = np.abs(dev[:, j] - ref[:, j]) / np.maximum(np.abs(ref[:, j]), 1e-300)
      assert rel.max() <= 6e-16, (j, rel.max())   # the device log: <= 2 ulp
      assert np.mean(dev[:, j] == ref[:, j]) > 0.98
    else:
      np.testing.assert_array_equal(dev[:, j], ref[:, j])


@pytest.mark.parametrize('name', sorted(_specs()))
def test_device_streams_equal_numpy_randomstate(name):
  spec = _specs()[name]
  n, t = 96, 37
  seeds = np.concatenate([[0, 1, 2 ** 32 - 1, 123456789],
                          np.arange(1000, 1000 + n - 4)])
  eng = _engine(spec, n, seeds)
  eng.legacy_replay(t)
  dev = eng.get_replay(0, t)
  thr = eng.get_replay(0, t, eng.stream_width() - 1)
  eng.close()
  ref = oracle.legacy_streams(spec, seeds, t)
  d = int(spec['dim'])
  normal = range(d) if spec['proposal']['kind'] == 'gauss' else ()
  _check(dev, ref, set(normal))
  np.testing.assert_array_equal(thr, dev[:, -1, :])


def test_device_streams_continue_across_calls():
  spec = _specs()['gauss5_permuted']
  n = 64
  seeds = np.arange(77, 77 + n)
  eng = _engine(spec, n, seeds)
  eng.legacy_replay(13)
  a = eng.get_replay(0, 13)
  eng.legacy_replay(24)
  b = eng.get_replay(0, 24)
  eng.close()
  ref = oracle.legacy_streams(spec, seeds, 37)
  _check(np.concatenate([a, b]), ref, set(range(5)))


def test_full_width_cfg2_replay_on_device_streams():
  from probayes_amd import Engine
  spec = oracle.golden_spec('diag10')
  n, t = 65536, 100
  seeds = np.arange(n) + 9_000_000
  eng = Engine(spec)
  eng.init_chains(np.zeros((n, 10)))
  eng.set_rng('replay')
  eng.seed_legacy(seeds)
  eng.legacy_replay(t)
  eng.alloc_trace(t, 1)
  eng.run(t)
  out = eng.trace()
  mom = eng.moments()
  eng.close()
  assert np.array_equal(mom['n_acc'], out['u'].sum(axis=1))
  pick = np.random.RandomState(11).choice(n, 192, replace=False)
  ref = oracle.run_mh(spec, np.zeros((192, 10)),
                      oracle.legacy_streams(spec, seeds[pick], t))
  assert np.array_equal(out['u'][pick], ref['u'])
  den = np.maximum(np.abs(ref['v_x']), 1.)
  assert np.max(np.abs(out['v_x'][pick] - ref['v_x']) / den) <= 1e-12
  den = np.maximum(np.abs(ref['v_p']), np.finfo(float).tiny)
  assert np.max(np.abs(out['v_p'][pick] - ref['v_p']) / den) <= 1e-12


@pytest.mark.parametrize('name', ['diag10', 'uniform10', 'randint_wide', 'gauss5_permuted'])
def test_device_streams_many_short_launches(name):
  """Launch boundaries at every phase of the LDS window and of the
  double-buffered state (mid-quad positions, block ends, pending refills):
  launches of 1, 2, 3, 5, ... steps in a row equal one RandomState stream,
  and so does one long launch spanning several 624-word blocks."""
  spec = _specs()[name]
  n = 80
  seeds = np.arange(5000, 5000 + n)
  sizes = [1, 2, 3, 5, 8, 13, 21, 34, 1, 1, 40]
  eng = _engine(spec, n, seeds)
  parts = []
  for t in sizes:
    eng.legacy_replay(t)
    parts.append(eng.get_replay(0, t))
  eng.close()
  total = sum(sizes)
  ref = oracle.legacy_streams(spec, seeds, total)
  d = int(spec['dim'])
  normal = set(range(d)) if spec['proposal']['kind'] == 'gauss' else set()
  _check(np.concatenate(parts), ref, normal)
  eng = _engine(spec, n, seeds)
  eng.legacy_replay(total)
  one = eng.get_replay(0, total)
  eng.close()
  _check(one, ref, normal)


@pytest.mark.parametrize('name', ['diag10', 'gauss5_permuted'])
def test_device_streams_long_drift(name):
  """Thousands of steps: the lanes of a wave drift hundreds of words apart
  in their streams, so the four-block generator's laggards bank twisted
  blocks (up to three ahead) while the leader sets the twist rounds, and
  launches start and end anywhere in a block; every chain still draws its
  own RandomState stream."""
  spec = _specs()[name]
  n = 96                                 # a full and a partial wavefront
  seeds = np.arange(77_000, 77_000 + n)
  sizes = [1000, 7, 1493]
  eng = _engine(spec, n, seeds)
  parts = []
  for t in sizes:
    eng.legacy_replay(t)
    parts.append(eng.get_replay(0, t))
  eng.close()
  ref = oracle.legacy_streams(spec, seeds, sum(sizes))
  _check(np.concatenate(parts), ref, set(range(int(spec['dim']))))
