"""The word-parallel legacy generator (pbh_legacy_wp.hip, the default for MH
streams of doubles; PBH_LEGACY_WP=0 keeps the chain-per-lane Mt4 generator):
one wavefront per chain, a whole MT block at a time, the polar method's
accept map by ballots and its attempt chains by table.

Checked here bit for bit against the chain-per-lane generator -- the same
values, the same order, the same cached deviate -- across launch splits that
start and end at every phase of a block, with the generator state handed
from one generator to the other in both directions, with a cached deviate
leading an even-d stream (the table path with has = 1), and at full cfg2
width.  tests/test_gpu_legacy.py checks the streams against NumPy's own
RandomState (the oracle) with the default (word-parallel) generator.
"""
import ctypes as _c

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

SPLITS = [1, 2, 3, 5, 8, 13, 21, 34, 1, 1, 40, 300, 7]


def _spec(name):
  if name == 'gauss5_permuted':
    s5 = oracle.golden_spec('diag10')
    s5.update(dim=5, names=['x{}'.format(i) for i in range(5)])
    s5['target'] = {'kind': 'diag_gauss', 'mu': np.zeros(5), 'sigma': np.ones(5)}
    s5['proposal'] = {'kind': 'gauss', 'loc': np.zeros(5), 'scale': np.ones(5),
                      'order': np.array([3, 0, 4, 1, 2], np.int32)}
    s5['ufun'] = np.zeros(5, np.int32)
    return s5
  if name == 'uniform10':
    su = oracle.golden_spec('diag10')
    su['proposal'] = {'kind': 'uniform', 'delta': np.full(10, 0.3)}
    return su
  if name == 'gauss1':
    s1 = oracle.golden_spec('diag10')
    s1.update(dim=1, names=['x'])
    s1['target'] = {'kind': 'diag_gauss', 'mu': np.zeros(1), 'sigma': np.ones(1)}
    s1['proposal'] = {'kind': 'gauss', 'loc': np.zeros(1), 'scale': np.ones(1)}
    s1['ufun'] = np.zeros(1, np.int32)
    return s1
  return oracle.golden_spec(name)


def _engine(monkeypatch, spec, seeds, wp):
  from probayes_amd import Engine
  monkeypatch.setenv('PBH_LEGACY_WP', '1' if wp else '0')
  eng = Engine(spec)
  eng.init_chains(np.zeros((len(seeds), int(spec['dim']))))
  eng.seed_legacy(seeds)
  return eng


def _streams(eng, sizes):
  parts = []
  for t in sizes:
    eng.legacy_replay(t)
    parts.append(eng.get_replay(0, t))
  return np.concatenate(parts)


def _set_legacy(eng, st):
  from probayes_amd import _lib
  _lib.call('pbh_set_legacy_state', eng._h,
            np.ascontiguousarray(st['key'], np.uint32).ctypes.data_as(_lib._u32p),
            np.ascontiguousarray(st['pos'], np.int32).ctypes.data_as(_lib._i32p),
            np.ascontiguousarray(st['has'], np.int32).ctypes.data_as(_lib._i32p),
            np.ascontiguousarray(st['gauss'], np.float64).ctypes.data_as(
                _c.POINTER(_c.c_double)))


def _same(a, b):
  nan = np.isnan(a)
  assert np.array_equal(nan, np.isnan(b))
  bad = np.argwhere(np.where(nan, 0., a) != np.where(nan, 0., b))
  assert not len(bad), 'first mismatches (step, draw, chain): {} of {}'.format(
      bad[:8].tolist(), len(bad))


NAMES = ['diag10', 'gmm2', 'mcmc_prob6', 'metrohast_norm1d', 'covrw5', 'uniform10',
         'gauss5_permuted', 'gauss1']


@pytest.mark.parametrize('name', NAMES)
def test_wp_streams_equal_chain_per_lane(monkeypatch, name):
  spec = _spec(name)
  n = 136                                   # two waves' worth and a ragged rest
  seeds = np.concatenate([[0, 1, 2 ** 32 - 1], np.arange(4000, 4000 + n - 3)])
  a = _engine(monkeypatch, spec, seeds, True)
  b = _engine(monkeypatch, spec, seeds, False)
  sa, sb = _streams(a, SPLITS), _streams(b, SPLITS)
  _same(sa, sb)
  # hand the state over in both directions and continue
  st_a, st_b = a._legacy_state(), b._legacy_state()
  assert np.array_equal(st_a['has'], st_b['has'])
  assert np.array_equal(st_a['gauss'], st_b['gauss'])
  _set_legacy(a, st_b)
  _set_legacy(b, st_a)
  _same(_streams(a, [9, 250]), _streams(b, [9, 250]))
  a.close()
  b.close()


def test_wp_even_d_with_a_leading_cached_deviate(monkeypatch):
  """An odd-d stream leaves the polar method's second deviate cached; handed
  to an even-d model every step then starts with it (the table path with a
  cached deviate leading each step and the last pair's second deviate
  cached for the next step)."""
  n = 72
  seeds = np.arange(31, 31 + n)
  odd = _engine(monkeypatch, _spec('gauss5_permuted'), seeds, False)
  odd.legacy_replay(3)                      # 15 normals: one cached
  st = odd._legacy_state()
  odd.close()
  assert st['has'].all()
  spec = _spec('diag10')
  out = []
  for wp in (True, False):
    eng = _engine(monkeypatch, spec, seeds, wp)
    _set_legacy(eng, st)
    out.append(_streams(eng, [1, 30, 2, 200]))
    fin = eng._legacy_state()
    assert fin['has'].all()
    out.append(fin['gauss'])
    eng.close()
  _same(out[0], out[2])
  assert np.array_equal(out[1], out[3])
  ref = oracle.legacy_streams(_spec('gauss5_permuted'), seeds, 3)   # sanity: odd stream
  assert ref.shape[0] == 3


def test_wp_full_width_equals_chain_per_lane(monkeypatch):
  spec = _spec('diag10')
  n = 65536
  seeds = np.arange(n) + 123
  a = _engine(monkeypatch, spec, seeds, True)
  b = _engine(monkeypatch, spec, seeds, False)
  for t in (250, 1):
    a.legacy_replay(t)
    b.legacy_replay(t)
    pick = np.random.RandomState(t).choice(n, 512, replace=False)
    ra = a.get_replay(0, t)[:, :, pick]
    rb = b.get_replay(0, t)[:, :, pick]
    _same(ra, rb)
  a.close()
  b.close()
