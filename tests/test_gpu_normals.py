"""The production Gibbs kernel's fp64 Box-Muller (pbh_device.h box_muller_tab:
log and sin/cos from LDS tables plus short polynomials)
against the libm form (box_muller: ocml log / sincospi) and against NumPy on
the host, on random and extreme Philox-like words."""
import numpy as np
import pytest

from probayes_amd import _lib

pytestmark = pytest.mark.gpu


def _normals(words):
  words = np.ascontiguousarray(words, np.uint32)
  n = words.shape[0]
  fast = np.empty((n, 2))
  ref = np.empty((n, 2))
  _lib.call('pbh_check_normals', 0, n, words.ctypes.data_as(_lib._u32p),
            fast.ctypes.data_as(_lib._dp), ref.ctypes.data_as(_lib._dp))
  return fast, ref


def _u01(a, b):
  return ((a >> 5).astype(np.float64) * 67108864.0 +
          (b >> 6).astype(np.float64)) / 9007199254740992.0


def test_fast_box_muller_matches_libm_and_numpy():
  rng = np.random.RandomState(3)
  n = 1 << 20
  w = rng.randint(0, 2 ** 32, (n, 4), dtype=np.uint64).astype(np.uint32)
  # extremes: u1 = 1 (r = 0), u1 = 2^-53 (largest r), u2 at quadrant edges
  w[:8, :2] = [[0, 0], [0xFFFFFFFF, 0xFFFFFFFF], [0xFFFFFFE0, 0xFFFFFFC0],
               [0, 64], [0x80000000, 0], [0x40000000, 0], [0xC0000000, 0],
               [1, 1]]
  w[8:16, 2:] = [[0, 0], [0x40000000, 0], [0x80000000, 0], [0xC0000000, 0],
                 [0x20000000, 0], [0x60000000, 0], [0xFFFFFFFF, 0xFFFFFFFF],
                 [0x3FFFFFFF, 0xFFFFFFFF]]
  fast, ref = _normals(w)
  scale = np.maximum(1.0, np.abs(ref))
  assert np.max(np.abs(fast - ref) / scale) < 4e-15
  u1 = 1.0 - _u01(w[:, 0], w[:, 1])
  u2 = _u01(w[:, 2], w[:, 3])
  r = np.sqrt(-2.0 * np.log(u1))
  host = np.stack([r * np.cos(2 * np.pi * u2), r * np.sin(2 * np.pi * u2)], 1)
  # NumPy rounds the angle 2 pi u2 before cos/sin: absolute error ~ r ulp
  assert np.max(np.abs(fast - host) / np.maximum(1.0, r)[:, None]) < 1e-14
  assert np.isfinite(fast).all()


def _normals64(words):
  words = np.ascontiguousarray(words, np.uint32)
  n = words.shape[0]
  fast = np.empty((n, 2))
  ref = np.empty((n, 2))
  _lib.call('pbh_check_normals64', 0, n, words.ctypes.data_as(_lib._u32p),
            fast.ctypes.data_as(_lib._dp), ref.ctypes.data_as(_lib._dp))
  return fast, ref


def _bm96_host(w):
  """bm96_pair's construction in NumPy (pbh_device.h): u1 = (k1 + 1/2)
  2^-52 from b[31:12]:a, the full-turn angle (J + c 2^-32) 2 pi / 1024 with
  J = b[11:2]."""
  w = w.astype(np.uint64)
  k1 = ((w[:, 1] >> 12) << 32) | w[:, 0]
  u1 = (k1.astype(np.float64) + 0.5) * 2.0 ** -52
  j = ((w[:, 1] >> 2) & 0x3FF).astype(np.float64)
  ang = (j + w[:, 2].astype(np.float64) * 2.0 ** -32) * (2 * np.pi / 1024)
  r = np.sqrt(-2.0 * np.log(u1))
  return np.stack([r * np.cos(ang), r * np.sin(ang)], 1), r


def _words96(rng, n):
  w = rng.randint(0, 2 ** 32, (n, 3), dtype=np.uint64).astype(np.uint32)
  # extremes: u1 at 2^-53 (largest r) and 1 - 2^-53 (r -> 0), the
  # mantissa's round-up to c = 1, angles at the table's rows 0, 255, 256 (a
  # quarter turn), 1023 and at a row's end
  w[0, :2] = [0, 0]
  w[1, :2] = [0xFFFFFFFF, 0xFFFFFFFF]
  w[2, :2] = [0, 0xFFF00000]
  w[3, :2] = [0xFFFFFFFF, 0xFFEFFFFF]
  w[4:10, 1] = (w[4:10, 1] & 0xFFFFF003) | (np.array([0, 255, 256, 1023, 512, 768],
                                                     np.uint32) << 2)
  w[4:10, 2] = [0, 0xFFFFFFFF, 0, 0xFFFFFFFF, 0, 1]
  return w


def test_bm64_normals_match_libm_and_numpy():
  """The production fp64 normals (bm96_pair: 1025-entry log table + degree-5
  log1p, rsq + Newton sqrt, 1024-entry full-turn sin/cos table) against the
  same construction through ocml's libm and through NumPy on the host:
  within a few ulp (absolute below |z| = 1, relative above)."""
  rng = np.random.RandomState(11)
  n = 1 << 20
  w = _words96(rng, n)
  fast, ref = _normals64(w)
  assert np.isfinite(fast).all()
  scale = np.maximum(1.0, np.abs(ref))
  assert np.max(np.abs(fast - ref) / scale) < 4e-15
  host, r = _bm96_host(w)
  assert np.max(np.abs(fast - host) / np.maximum(1.0, r)[:, None]) < 1e-14
  # r near 0 keeps relative accuracy (u1 -> 1: ln c = 0 exactly)
  small = r < 1e-3
  assert small.any()
  rel = np.abs(np.hypot(fast[small, 0], fast[small, 1]) / r[small] - 1)
  assert rel.max() < 1e-14
  # the largest radius: u1 = 2^-53
  assert abs(np.hypot(*fast[0]) - np.sqrt(2 * 53 * np.log(2.0))) < 1e-13


def test_bm64_normals_are_standard_normal():
  """Distribution of the production normals: moments, tail mass beyond the
  fp32 form's 5.77 sigma cut, and a Kolmogorov-Smirnov test."""
  import scipy.stats
  rng = np.random.RandomState(5)
  n = 1 << 22
  w = rng.randint(0, 2 ** 32, (n, 3), dtype=np.uint64).astype(np.uint32)
  fast, _ = _normals64(w)
  z = fast.reshape(-1)
  m = z.size
  assert abs(z.mean()) < 5 / np.sqrt(m)
  assert abs(z.var() - 1) < 5 * np.sqrt(2 / m)
  assert abs(scipy.stats.skew(z)) < 5 * np.sqrt(6 / m)
  assert abs(scipy.stats.kurtosis(z)) < 5 * np.sqrt(24 / m)
  # P(|z| > 4) = 6.33e-5: binomial 5-sigma band
  p4 = 2 * scipy.stats.norm.sf(4)
  k4 = np.sum(np.abs(z) > 4)
  assert abs(k4 - m * p4) < 5 * np.sqrt(m * p4)
  assert scipy.stats.kstest(z[:1 << 21], 'norm').pvalue > 1e-3
  # the two normals of a pair are uncorrelated, and so are their squares
  assert abs(np.corrcoef(fast[:, 0], fast[:, 1])[0, 1]) < 5 / np.sqrt(n)
  assert abs(np.corrcoef(fast[:, 0] ** 2, fast[:, 1] ** 2)[0, 1]) < 5 / np.sqrt(n)
  # the angle is uniform over the full turn: equal mass in the 8 octants
  oct_ = np.floor((np.arctan2(fast[:, 1], fast[:, 0]) + np.pi) / (np.pi / 4)).astype(int) % 8
  cnt = np.bincount(oct_, minlength=8)
  assert scipy.stats.chisquare(cnt).pvalue > 1e-3
