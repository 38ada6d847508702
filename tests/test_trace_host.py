"""Host-side trace handling (no GPU): the accept words' unpacking into the
u [N, T] array the summaries read (probayes_amd.engine.unpack_accept),
against the per-record unpack it replaced, at ragged chain counts."""
import numpy as np
import pytest

from probayes_amd.engine import unpack_accept


@pytest.mark.parametrize('n,count', [(1, 5), (63, 7), (64, 3), (65, 9), (1000, 13),
                                     (4097, 2), (65536, 20)])
def test_unpack_accept_equals_per_record_unpack(n, count):
  rng = np.random.default_rng(n * 31 + count)
  W = (n + 63) // 64
  acc = (rng.integers(0, 2 ** 63, size=(count, W), dtype=np.uint64) * np.uint64(2) +
         rng.integers(0, 2, size=(count, W), dtype=np.uint64))
  bits = np.unpackbits(acc.view(np.uint8).reshape(count, W * 8), axis=1,
                       bitorder='little')[:, :n]
  u = unpack_accept(acc, n)
  assert u.shape == (n, count) and u.dtype == np.uint8 and u.flags.c_contiguous
  np.testing.assert_array_equal(u, bits.T)
  # chain c, record t is bit c % 64 of word c // 64
  t, c = count - 1, n - 1
  assert u[c, t] == (int(acc[t, c // 64]) >> (c % 64)) & 1
