"""The production acceptance filter (pbh_device.h accept_filter) must make
exactly the decisions of the reference's ratio form (sp_utils.py:40-64,
pscales.py:56-65,219-236) whenever it does not defer to the exact fallback,
and must defer rarely.  Checked on device through pbh_check_accept on
random and adversarial (lp, lp', t) triples, including t placed within 1e-7
of the acceptance probability, the |lp| > 700 clamp regime, NaN and inf."""
import ctypes

import numpy as np
import pytest

from probayes_amd import _lib

pytestmark = pytest.mark.gpu


def _check(lp, lpp, t0, t1, lin=0):
  n = len(lp)
  lp = np.ascontiguousarray(lp, np.float64)
  lpp = np.ascontiguousarray(lpp, np.float64)
  t0 = np.ascontiguousarray(t0, np.uint32)
  t1 = np.ascontiguousarray(t1, np.uint32)
  out = np.zeros(n, np.uint8)
  _lib.call('pbh_check_accept', 0, n, lp.ctypes.data_as(_lib._dp),
            lpp.ctypes.data_as(_lib._dp), t0.ctypes.data_as(_lib._u32p),
            t1.ctypes.data_as(_lib._u32p), lin, out.ctypes.data_as(_lib._u8p))
  return (out & 1).astype(bool), (out & 2).astype(bool), (out & 4).astype(bool)


def _u01(t0, t1):
  return ((t0 >> 5).astype(np.float64) * 67108864.0 +
          (t1 >> 6).astype(np.float64)) / 9007199254740992.0


def _words_near(p, rng, rel=1e-7):
  """(t0, t1) whose u01 lies within rel of p (p in (0, 1))."""
  t = np.clip(p * (1 + rng.uniform(-rel, rel, p.shape)), 0, 1 - 2 ** -53)
  k = np.floor(t * 2.0 ** 53).astype(np.uint64)
  t0 = ((k >> np.uint64(26)) << np.uint64(5)).astype(np.uint32)
  t1 = ((k & np.uint64((1 << 26) - 1)) << np.uint64(6)).astype(np.uint32)
  return t0, t1


def test_filter_decisions_equal_exact_ratio_form():
  rng = np.random.RandomState(11)
  n = 1 << 21
  lp = rng.uniform(-60., 5., n)
  d = np.concatenate([rng.normal(0, 1, n // 2), rng.normal(0, 20, n - n // 2)])
  lpp = lp + d
  t0 = rng.randint(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
  t1 = rng.randint(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
  ex, decided, fast = _check(lp, lpp, t0, t1)
  assert np.array_equal(fast[decided], ex[decided])
  assert (~decided).mean() < 1e-4, (~decided).mean()
  # the exact device decision agrees with NumPy's ratio form away from ties
  s = np.minimum(np.exp(lpp) / np.maximum(np.exp(lp), 2.2250738585072014e-308), 1.)
  t = _u01(t0, t1)
  clear = np.abs(s - t) > 1e-12 * np.maximum(s, t)
  assert np.array_equal(ex[clear], (s >= t)[clear])


def test_filter_adversarial_boundaries_and_regimes():
  rng = np.random.RandomState(12)
  n = 1 << 20
  lp = rng.uniform(-300., 300., n)
  d = -rng.exponential(3., n)
  lpp = lp + d
  p = np.exp(d)                         # the acceptance probability
  t0, t1 = _words_near(p, rng)          # t within 1e-7 of it
  ex, decided, fast = _check(lp, lpp, t0, t1)
  assert np.array_equal(fast[decided], ex[decided])
  assert (~decided).mean() > 0.5        # the band makes these defer

  # clamp / underflow regime (|lp| > 700), specials, extreme words
  lps = np.array([-800., -750., -710., 700.5, 710., 800., -1e308, 0., 0.,
                  np.nan, 0., np.inf, -np.inf, 5., -5., 0.])
  lpps = np.array([-801., -749., -700., 701., 709., 900., -1e308, np.nan,
                   np.inf, 0., -np.inf, 0., 0., 5., -5. - 1e-15, 1e-300])
  m = len(lps)
  reps = 4096
  LP = np.tile(lps, reps)
  LPP = np.tile(lpps, reps)
  T0 = rng.randint(0, 2 ** 32, m * reps, dtype=np.uint64).astype(np.uint32)
  T1 = rng.randint(0, 2 ** 32, m * reps, dtype=np.uint64).astype(np.uint32)
  T0[:m], T1[:m] = 0, 0
  T0[m:2 * m], T1[m:2 * m] = 0xFFFFFFFF, 0xFFFFFFFF
  ex, decided, fast = _check(LP, LPP, T0, T1)
  assert np.array_equal(fast[decided], ex[decided])
  out_of_range = ~((np.abs(LP) <= 700) & (np.abs(LPP) <= 700))
  assert not decided[out_of_range].any()


def test_filter_defers_for_linear_pscale():
  rng = np.random.RandomState(13)
  n = 4096
  lp = rng.uniform(0.1, 1., n)
  lpp = rng.uniform(0.1, 1., n)
  t0 = rng.randint(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
  t1 = rng.randint(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
  ex, decided, _ = _check(lp, lpp, t0, t1, lin=1)
  assert not decided.any()
  s = np.minimum(lpp / lp, 1.)
  assert np.array_equal(ex, s >= _u01(t0, t1))
