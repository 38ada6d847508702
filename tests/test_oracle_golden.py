"""Pins the CPU oracle to the reference: every golden workload recorded by
tools/gen_golden.py (which ran probayes 0.0.8 itself) must be reproduced
BIT-FOR-BIT by oracle.run_mh / oracle.run_gibbs on the same legacy streams."""
import numpy as np
import pytest

import oracle
from oracle.workloads import golden_init


@pytest.mark.parametrize('name', sorted(oracle.WORKLOADS))
def test_oracle_matches_reference_bitwise(name):
  g = oracle.load_golden(name)
  spec = oracle.golden_spec(name, g)
  n, t = g['v_x'].shape[:2]
  streams = oracle.legacy_streams(spec, g['seeds'], t)
  run = oracle.run_gibbs if spec['scores'] == 'gibbs' else oracle.run_mh
  out = run(spec, golden_init(name, n), streams)
  keys = ['v_x', 'v_p', 'p_x', 'p_p', 'u']
  if spec['scores'] != 'gibbs':
    keys += ['s', 't']
  for k in keys:
    np.testing.assert_array_equal(out[k], g[k], err_msg='{}:{}'.format(name, k))


def test_golden_fixture_metadata():
  for name in oracle.WORKLOADS:
    g = oracle.load_golden(name)
    assert g['meta']['name'] == name
    assert g['meta']['generator'] == 'tools/gen_golden.py'
    assert len(g['seeds']) == g['v_x'].shape[0]


def test_streams_layout_and_determinism():
  spec = oracle.golden_spec('diag10')
  a = oracle.legacy_streams(spec, [5, 6], 4)
  b = oracle.legacy_streams(spec, [5, 6], 4)
  assert a.shape == (4, 11, 2)
  np.testing.assert_array_equal(a, b)
  rs = np.random.RandomState(6)
  z = rs.standard_normal(10)
  u = rs.random_sample()
  np.testing.assert_array_equal(a[0, :10, 1], z)
  assert a[0, 10, 1] == u


@pytest.mark.parametrize('name', sorted(oracle.workloads.SEGMENTED))
def test_oracle_consecutive_samplers(name):
  """tools/gen_golden.py ran several samplers on ONE process (same init,
  NumPy's global stream continuing): each starts at the RF's current cycle
  phase (rf.py:446-452), which the oracle takes as step0 / cond_mod."""
  from oracle.workloads import SEGMENTED, golden_params, WORKLOADS
  g = oracle.load_golden(name)
  base, segs = SEGMENTED[name], [int(s) for s in g['segments']]
  n, T = g['v_x'].shape[:2]
  assert sum(segs) == T and len(segs) > 1
  parts, t0 = [], 0
  if base == 'gibbs_linreg':
    from oracle.linreg import linreg_streams, run_linreg
    x, y = g['param_x_obs'], g['param_y_obs']
    init = np.tile(g['param_init'], (n, 1))
    z = linreg_streams(g['seeds'], T, len(x))
    for L in segs:
      parts.append(run_linreg(x, y, init, z[t0:t0 + L], cond_mod=t0 % 3))
      t0 += L
  else:
    spec = WORKLOADS[base](golden_params(g))
    st = oracle.legacy_streams(spec, g['seeds'], T)
    for L in segs:
      parts.append(oracle.run_gibbs(spec, golden_init(base, n),
                                    st[t0:t0 + L], step0=t0))
      t0 += L
  for k in ('v_x', 'v_p'):
    np.testing.assert_array_equal(np.concatenate([p[k] for p in parts], 1),
                                  g[k], err_msg=k)
