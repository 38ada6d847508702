"""Covariance-matrix random walk on the GPU.

RF.set_tran(ndarray) installs chol(cov) as the RF's tfun (rf.py:210-220) and
RF.eval_delta multiplies every base delta by it (rf.py:340-354).  The golden
workloads covrw2 / covrw5 (recorded from the reference by tools/gen_golden.py)
run through test_gpu_parity.test_replay_matches_reference_golden; here:
  * the delta law: in PHILOX_F64 mode the recorded proposal steps p_x - x
    have covariance step^2 cov (the check of examples/cov/delta_cov_xyz.py);
  * production Philox posterior of a 10-dim target under a covariance RW
    within Monte-Carlo error, and equal to the reference-arithmetic mode;
  * replay parity at a larger chain count and odd dimension.
"""
import numpy as np
import pytest

import oracle
from oracle.workloads import golden_init

pytestmark = pytest.mark.gpu


def _engine(spec):
  from probayes_amd import Engine
  return Engine(spec)


def _cov10():
  rs = np.random.RandomState(77)
  A = rs.normal(size=(10, 10))
  return A.dot(A.T) / 10 + 0.3 * np.eye(10)


def _spec10(step=0.25):
  spec = oracle.golden_spec('diag10')
  spec['proposal']['scale'] = np.full(10, step)
  spec['proposal']['tfun'] = np.linalg.cholesky(_cov10())
  return spec


def test_delta_covariance_is_step2_cov():
  spec = _spec10()
  n, t = 4096, 64
  eng = _engine(spec)
  eng.init_chains(np.zeros((n, 10)))
  eng.set_rng('philox_f64', seed=5)
  eng.alloc_trace(t, 1, debug=True)
  eng.run(t)
  tr = eng.trace()
  eng.close()
  prev = np.concatenate([np.zeros((n, 1, 10)), tr['v_x'][:, :-1]], axis=1)
  steps = (tr['p_x'] - prev).reshape(-1, 10)
  emp = np.cov(steps.T)
  want = 0.25 ** 2 * _cov10()
  scale = np.sqrt(np.outer(np.diag(want), np.diag(want)))
  # 262 144 draws: the correlation estimates are good to ~0.01
  assert np.max(np.abs(emp - want) / scale) < 0.03, np.max(np.abs(emp - want) / scale)


@pytest.mark.parametrize('mode', ['philox', 'philox_f64'])
def test_production_posterior_under_covariance_rw(mode):
  # chains start at exact draws from the target, so any deviation of the
  # moments is a bias of the kernel, not an unfinished burn-in (the
  # correlated proposal mixes slowly along cov10's small eigen-directions)
  spec = _spec10()
  n, burn, t = 8192, 100, 900
  mu, sg = spec['target']['mu'], spec['target']['sigma']
  eng = _engine(spec)
  eng.init_chains(mu + sg * np.random.RandomState(3).standard_normal((n, 10)))
  eng.set_rng(mode, seed=11)
  eng.run(burn)
  eng.reset_moments()
  eng.run(t)
  mom = eng.moments()
  eng.close()
  steps = mom['n_steps']
  mean = mom['sum'].sum(0) / (n * steps)
  var = mom['sumsq'].sum(0) / (n * steps) - mean ** 2
  assert np.all(np.abs(mean - mu) < 0.06 * sg), (mean, mu)
  assert np.all(np.abs(var / sg ** 2 - 1) < 0.06), var / sg ** 2
  acc = mom['n_acc'].sum() / (n * steps)
  assert 0.05 < acc < 0.9, acc


@pytest.mark.parametrize('name,n,t', [('covrw5', 333, 200), ('covrw2', 1000, 200)])
def test_covariance_rw_replay_vs_oracle(name, n, t):
  spec = oracle.golden_spec(name)
  seeds = np.arange(60000, 60000 + n)
  streams = oracle.legacy_streams(spec, seeds, t)
  init = golden_init(name, n)
  ref = oracle.run_mh(spec, init, streams)
  eng = _engine(spec)
  eng.init_chains(init)
  eng.set_rng('replay')
  eng.upload_replay(streams)
  eng.alloc_trace(t, 1, debug=True)
  eng.run(t)
  out = eng.trace()
  eng.close()
  assert int(np.sum(out['u'] != ref['u'])) == 0
  den = np.maximum(np.abs(ref['p_x']), 1.)
  assert np.max(np.abs(out['p_x'] - ref['p_x']) / den) <= 1e-12
  den = np.maximum(np.abs(ref['v_p']), np.finfo(float).tiny)
  assert np.max(np.abs(out['v_p'] - ref['v_p']) / den) <= 1e-12
