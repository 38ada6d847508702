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
