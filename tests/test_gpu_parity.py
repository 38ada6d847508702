"""GPU parity: the HIP engine (through the C-ABI) against the oracle/reference.

Replay mode feeds the kernels the reference's own legacy-MT19937 streams, so
every golden workload must reproduce the reference traces step for step:
  * accept decisions u: identical (0 flips);
  * states and (log-)probabilities: relative error <= 1e-12 per step
    (device exp/log/ndtri differ from glibc/NumPy SIMD by ulps; the
    tolerance is SURVEY.md §7 step 4's);
  * posterior moments over the traces: <= 1e-6 relative (north star).
Philox mode (production RNG) is checked statistically and by invariants.
"""
import numpy as np
import pytest

import oracle
from oracle.workloads import golden_init

pytestmark = pytest.mark.gpu

RTOL = 1e-12


def _engine(spec):
  from probayes_amd import Engine
  return Engine(spec)


def _rel_err(a, b, floor=np.finfo(float).tiny):
  """max |a - b| / max(|b|, floor); states use floor 1 (absolute error near
  0, relative error elsewhere), probabilities are purely relative."""
  a, b = np.asarray(a, float), np.asarray(b, float)
  both_nan = np.isnan(a) & np.isnan(b)
  same = (a == b) | both_nan
  den = np.maximum(np.abs(b), floor)
  err = np.where(same, 0., np.abs(a - b) / den)
  return float(err.max()) if err.size else 0.


def _run_replay(spec, init, streams, debug=True):
  T = streams.shape[0]
  eng = _engine(spec)
  eng.init_chains(init)
  eng.set_rng('replay')
  eng.upload_replay(streams)
  eng.alloc_trace(T, 1, debug=debug)
  eng.run(T)
  out = eng.trace()
  mom = eng.moments()
  eng.close()
  return out, mom


@pytest.mark.parametrize('name', sorted(oracle.WORKLOADS))
def test_replay_matches_reference_golden(name):
  g = oracle.load_golden(name)
  spec = oracle.golden_spec(name, g)
  n, t = g['v_x'].shape[:2]
  streams = oracle.legacy_streams(spec, g['seeds'], t)
  out, mom = _run_replay(spec, golden_init(name, n), streams)
  flips = int(np.sum(out['u'] != g['u']))
  assert flips == 0, '{}: {} accept flips'.format(name, flips)
  assert _rel_err(out['v_x'], g['v_x'], 1.) <= RTOL
  assert _rel_err(out['v_p'], g['v_p']) <= RTOL
  assert _rel_err(out['p_x'], g['p_x'], 1.) <= RTOL
  assert _rel_err(out['p_p'], g['p_p']) <= RTOL
  if spec['scores'] != 'gibbs':
    assert _rel_err(out['s'], g['s']) <= 1e-10
  # in-kernel moments == moments of the recorded trace
  np.testing.assert_allclose(mom['sum'], g['v_x'].sum(axis=1), rtol=1e-9,
                             atol=1e-9)
  assert np.array_equal(mom['n_acc'], g['u'].sum(axis=1))


@pytest.mark.parametrize('name,n,t', [('diag10', 1024, 400),
                                      ('metrohast_norm1d', 256, 400),
                                      ('gibbs8', 512, 256),
                                      ('gmm2', 1024, 400)])
def test_replay_posterior_moments_vs_oracle(name, n, t):
  """Posterior moments of GPU replay runs vs the oracle: 1e-6 relative."""
  spec = oracle.golden_spec(name)
  seeds = np.arange(50000, 50000 + n)
  streams = oracle.legacy_streams(spec, seeds, t)
  init = golden_init(name, n)
  run = oracle.run_gibbs if spec['scores'] == 'gibbs' else oracle.run_mh
  ref = run(spec, init, streams)
  out, _ = _run_replay(spec, init, streams, debug=False)
  flips = np.sum(out['u'] != ref['u'])
  assert flips <= max(1, n * t // 10 ** 6), flips
  for k in ('v_x',):
    m_ref, m_gpu = ref[k].mean(axis=1), out[k].mean(axis=1)
    sd = ref[k].std(axis=1)
    den = np.maximum(np.abs(m_ref), sd)
    assert np.max(np.abs(m_gpu - m_ref) / den) <= 1e-6
    v_ref, v_gpu = ref[k].var(axis=1), out[k].var(axis=1)
    assert np.max(np.abs(v_gpu - v_ref) / np.maximum(v_ref, 1e-300)) <= 1e-6


def _diag10_spec():
  return oracle.golden_spec('diag10')


@pytest.mark.parametrize('mode', ['philox', 'philox_f64', 'xoshiro'])
def test_philox_diag10_statistics_and_invariants(mode):
  """cfg2 model in production (Philox) mode: the posterior matches the
  target within Monte-Carlo error; traces are deterministic and invariant to
  how chains are sharded (global chain ids key the RNG)."""
  spec = _diag10_spec()
  n, t = 8192, 1000
  mu, sg = spec['target']['mu'], spec['target']['sigma']
  # chains start IN the target (exact draws), so every step is a draw from
  # it: no burn-in bias, and the chains are independent
  init = mu + sg * np.random.RandomState(77).standard_normal((n, 10))
  eng = _engine(spec)
  eng.init_chains(init)
  eng.set_rng(mode, seed=1234)
  eng.run(t)
  mom = eng.moments()
  eng.close()
  steps = mom['n_steps']
  # Monte-Carlo standard errors from the spread of the per-chain averages
  # (independent chains: MCSE = sd(chain means) / sqrt(n), which carries the
  # autocorrelation of each chain)
  m_c = mom['sum'] / steps                   # [n, d]
  q_c = mom['sumsq'] / steps
  mean, mcse_m = m_c.mean(0), m_c.std(0) / np.sqrt(n)
  assert np.all(np.abs(mean - mu) <= 5 * mcse_m), ((mean - mu) / mcse_m)
  # E[x^2] = mu^2 + sigma^2, its MCSE likewise
  q, mcse_q = q_c.mean(0), q_c.std(0) / np.sqrt(n)
  assert np.all(np.abs(q - (mu ** 2 + sg ** 2)) <= 5 * mcse_q), \
      ((q - mu ** 2 - sg ** 2) / mcse_q)
  # the 5-MCSE band on the means is tighter than round 1's 5%-of-sigma bound
  assert np.all(5 * mcse_m < 0.05 * sg)
  acc = mom['n_acc'].sum() / (n * steps)
  assert 0.05 < acc < 0.6

  # determinism + sharding invariance on a short run with a trace
  def run(n0, n1, spl=17):
    e = _engine(spec)
    e.init_chains(np.zeros((n1 - n0, 10)), chain_offset=n0)
    e.set_rng(mode, seed=99)
    e.alloc_trace(50, 1)
    e.run(50, steps_per_launch=spl)
    tr = e.trace()
    e.close()
    return tr
  full = run(0, 4096)
  again = run(0, 4096, spl=0)          # one launch == three launches
  lo, hi = run(0, 2048), run(2048, 4096)
  np.testing.assert_array_equal(full['v_x'], again['v_x'])
  np.testing.assert_array_equal(full['v_x'][:2048], lo['v_x'])
  np.testing.assert_array_equal(full['v_x'][2048:], hi['v_x'])
  np.testing.assert_array_equal(full['u'][2048:], hi['u'])


def test_thinning_and_launch_split_equivalence():
  spec = oracle.golden_spec('gmm2')
  n, t = 300, 60          # ragged: n not a multiple of 64
  seeds = np.arange(7, 7 + n)
  streams = oracle.legacy_streams(spec, seeds, t)
  init = golden_init('gmm2', n)
  ref = oracle.run_mh(spec, init, streams)
  eng = _engine(spec)
  eng.init_chains(init)
  eng.set_rng('replay')
  eng.upload_replay(streams)
  eng.alloc_trace(t // 3, 3)
  eng.run(t, steps_per_launch=7)
  tr = eng.trace()
  eng.close()
  assert tr['v_x'].shape == (n, t // 3, 2)
  assert _rel_err(tr['v_x'], ref['v_x'][:, 2::3], 1.) <= RTOL
  assert np.array_equal(tr['u'], ref['u'][:, 2::3])


def test_engine_errors_are_loud():
  from probayes_amd._lib import PbhError
  spec = _diag10_spec()
  eng = _engine(spec)
  with pytest.raises(PbhError):
    eng.run(5)                      # no chains yet
  eng.init_chains(np.zeros((64, 10)))
  eng.set_rng('replay')
  with pytest.raises(PbhError):
    eng.run(5)                      # replay without a stream
  eng.set_rng('philox', 1)
  eng.alloc_trace(4, 1)
  with pytest.raises(PbhError):
    eng.run(5)                      # trace capacity exceeded
  eng.run(4)
  assert eng.trace_len() == 4
  eng.close()


def test_rccl_single_rank_allgather_and_max():
  """The engine's RCCL path (one rank: the GPU box has one card): the stats
  gather returns the engine's moments, the device ESS rows and the count."""
  from probayes_amd import Engine
  spec = _diag10_spec()
  eng = Engine(spec)
  eng.init_chains(np.zeros((1000, 10)))
  eng.set_rng('philox', 3)
  eng.alloc_trace(40, 1)
  eng.run(40)
  eng.rccl_init(0, 1, Engine.rccl_unique_id())
  g = eng.rccl_allgather_stats()
  assert np.isnan(g['ess']).all()          # no pbh_trace_ess yet
  m = eng.moments()
  ess = eng.trace_ess(10)
  g = eng.rccl_allgather_stats()
  assert list(g['counts']) == [1000]
  np.testing.assert_array_equal(g['sum'], m['sum'])
  np.testing.assert_array_equal(g['sumsq'], m['sumsq'])
  np.testing.assert_array_equal(g['n_acc'], m['n_acc'])
  np.testing.assert_array_equal(g['ess'], ess)
  assert eng.rccl_allreduce_max(2.5) == 2.5
  eng.close()


@pytest.mark.parametrize('step', ['1', '2', '3'])
def test_rccl_gather_local_failure_is_returned_after_the_collectives(monkeypatch, step):
  """PBH_FAULT_GATHER=0:step makes this rank fail step `step` of
  pbh_rccl_allgather_stats locally: the call still enters every agreement
  (so no peer would wait) and returns the error; the engine and its
  communicator stay usable."""
  from probayes_amd import Engine
  from probayes_amd._lib import PbhError
  eng = Engine(_diag10_spec())
  eng.init_chains(np.zeros((300, 10)))
  eng.set_rng('philox', 3)
  eng.alloc_trace(8, 1)
  eng.run(8)
  eng.rccl_init(0, 1, Engine.rccl_unique_id())
  monkeypatch.setenv('PBH_FAULT_GATHER', '0:' + step)
  with pytest.raises(PbhError, match='could not take part'):
    eng.rccl_allgather_stats()
  monkeypatch.delenv('PBH_FAULT_GATHER')
  g = eng.rccl_allgather_stats()
  assert list(g['counts']) == [300]
  assert eng.rccl_allreduce_max(1.5) == 1.5
  eng.close()


def _ess_ips(x):
  """scripts/bench_workloads.py's host estimator (FFT autocorrelation)."""
  n, t = x.shape
  xc = x - x.mean(axis=1, keepdims=True)
  f = np.fft.rfft(xc, n=2 * t, axis=1)
  ac = np.fft.irfft(f * np.conj(f), axis=1)[:, :t]
  ac /= np.maximum(ac[:, :1], 1e-300)
  m = (t - 1) // 2
  pairs = ac[:, 1:2 * m + 1:2] + ac[:, 2:2 * m + 2:2]
  neg = pairs <= 0
  first = np.where(neg.any(axis=1), neg.argmax(axis=1), m)
  keep = np.arange(m)[None, :] < first[:, None]
  s = np.sum(np.where(keep, pairs, 0.), axis=1)
  return t / np.maximum(1.0 + 2.0 * s, 1e-12), pairs, first


@pytest.mark.parametrize('fft', ['2', '3', '1', '0'])
@pytest.mark.parametrize('name,n,t,burn,scale', [('gmm2', 2000, 600, 100, None),
                                                 ('diag10', 300, 257, 7, None),
                                                 ('gmm2', 33, 2100, 40, None),
                                                 # odd d n: unaligned series pairs
                                                 ('mcmc_prob2', 33, 300, 10, None),
                                                 ('bound_list3', 33, 300, 10, None),
                                                 # the FFT kernels' edges: exactly
                                                 # 2 048 records (half the 4 096
                                                 # points), 1 536 (the 2 048-point
                                                 # form's last length), 1 537, and
                                                 # 13 records
                                                 ('gmm2', 64, 2058, 10, None),
                                                 ('gmm2', 64, 1546, 10, None),
                                                 ('gmm2', 64, 1547, 10, None),
                                                 ('diag10', 40, 23, 10, None),
                                                 # cfg5's record count: ~1 % of the
                                                 # pairs need lags past 548
                                                 ('gmm2', 2000, 2000, 500, None),
                                                 # slow mixing: most pairs' scans
                                                 # run past the 2 048-point form's
                                                 # exact lags (its fallback list)
                                                 ('gmm2', 300, 1400, 100, 0.05),
                                                 ('diag10', 65, 1300, 10, 0.02)])
def test_device_ess_and_trace_stats_match_host(monkeypatch, name, n, t, burn, scale, fft):
  """pbh_trace_ess (on-device initial positive sequence: the 2 048-point FFT
  kernel with the 4 096-point one for the pairs whose scan leaves its exact
  lags (PBH_ESS_FFT=2, the default), the 4 096-point kernel alone (1), or the
  direct-sum kernel (0); more than 2 048 records always take the direct sums)
  equals the host FFT estimator on the same trace within 1e-9 wherever the
  sequence's stopping pair is not within rounding of zero; pbh_trace_stats
  equals the host sums of the trace."""
  from probayes_amd import Engine
  monkeypatch.setenv('PBH_ESS_FFT', fft)
  spec = oracle.golden_spec(name)
  if scale is not None:
    spec['proposal']['scale'] = np.full_like(spec['proposal']['scale'], scale)
  eng = Engine(spec)
  eng.init_chains(golden_init(name, n))
  eng.set_rng('philox', seed=17)
  eng.set_collect(moments=False)
  eng.alloc_trace(t, 1)
  eng.run(t, steps_per_launch=100)
  tr = eng.trace()
  dev = eng.trace_ess(burn)
  assert np.array_equal(dev, eng.trace_ess(burn))   # the fallback list resets
  st = eng.trace_stats(burn)
  eng.close()
  x = tr['v_x'][:, burn:]
  np.testing.assert_allclose(st['sum'], x.sum(1), rtol=1e-12, atol=1e-12)
  np.testing.assert_allclose(st['sumsq'], (x * x).sum(1), rtol=1e-12, atol=1e-12)
  assert np.array_equal(st['n_acc'], tr['u'][:, burn:].sum(1))
  for k in range(x.shape[2]):
    host, pairs, first = _ess_ips(x[:, :, k])
    # chains whose decisive pair (the first non-positive one) is within
    # rounding of 0 may stop one pair apart between the two summations
    m = pairs.shape[1]
    dec = np.abs(pairs[np.arange(len(first)), np.minimum(first, m - 1)])
    # a series that never moved (short traces) has no autocovariance: what
    # is left after centring is the mean's rounding, which differs between
    # the two summation orders -- the estimate is undefined; finite and
    # within (0, T] on the device is all that is asked
    flat = np.ptp(x[:, :, k], axis=1) == 0
    assert np.all((dev[flat, k] > 0) & (dev[flat, k] <= x.shape[1] + 1e-9))
    clear = (dec > 1e-9) & ~flat
    assert (~clear & ~flat).sum() <= max(1, 0.01 * clear.size)
    rel = np.abs(dev[clear, k] / host[clear] - 1)
    assert rel.max() < 1e-9, rel.max()


@pytest.mark.parametrize('n', [32, 100])
def test_lane_pair_kernel_replay_matches_reference(n):
  """The cfg2 form without debug records runs the lane-pair kernel (one chain
  per lanes l, l+32); it must reproduce the reference golden chains too,
  including ragged chain counts."""
  g = oracle.load_golden('diag10')
  spec = oracle.golden_spec('diag10', g)
  t = g['v_x'].shape[1]
  seeds = np.concatenate([g['seeds'], np.arange(90000, 90000 + n - 32)])
  streams = oracle.legacy_streams(spec, seeds, t)
  out, mom = _run_replay(spec, golden_init('diag10', n), streams, debug=False)
  ref = oracle.run_mh(spec, golden_init('diag10', n), streams)
  assert np.array_equal(out['u'], ref['u'])
  assert np.array_equal(out['u'][:32], g['u'])
  assert _rel_err(out['v_x'], ref['v_x'], 1.) <= RTOL
  assert _rel_err(out['v_p'], ref['v_p']) <= RTOL
  assert np.array_equal(mom['n_acc'], ref['u'].sum(axis=1))
  np.testing.assert_allclose(mom['sum'], ref['v_x'].sum(axis=1), rtol=1e-9,
                             atol=1e-9)


def test_full_size_cfg2_replay_parity():
  """BASELINE cfg2 at full width (65 536 chains): the GPU runs the
  reference's own per-chain legacy streams; 256 sampled chains must match
  the oracle step for step, and size-independent invariants hold for all
  chains (trace accept bits == in-kernel accept counts, trace sums ==
  in-kernel moments, every chain moved on step 1)."""
  from probayes_amd.replay import legacy_streams_parallel
  spec = oracle.golden_spec('diag10')
  n, t = 65536, 120
  seeds = np.arange(n, dtype=np.int64) + 7_000_000
  streams = legacy_streams_parallel(spec, t, seeds, processes=16)
  out, mom = _run_replay(spec, np.zeros((n, 10)), streams, debug=False)
  assert np.array_equal(mom['n_acc'], out['u'].sum(axis=1))
  np.testing.assert_allclose(mom['sum'], out['v_x'].sum(axis=1), rtol=1e-12,
                             atol=1e-9)
  assert out['u'][:, 0].all()
  pick = np.random.RandomState(5).choice(n, 256, replace=False)
  ref = oracle.run_mh(spec, np.zeros((256, 10)), streams[:, :, pick])
  assert np.array_equal(out['u'][pick], ref['u'])
  assert _rel_err(out['v_x'][pick], ref['v_x'], 1.) <= RTOL
  assert _rel_err(out['v_p'][pick], ref['v_p']) <= RTOL


@pytest.mark.parametrize('name', ['gibbs8', 'gibbs_norm2d', 'gibbs_sweep2'])
def test_gibbs_density_mfma_matches_valu(name, monkeypatch):
  """The Gibbs v.prob quadratic form on MFMA (v_mfma_f64_16x16x4_f64) and on
  the VALU agree to fp64 rounding and both match the reference."""
  g = oracle.load_golden(name)
  spec = oracle.golden_spec(name, g)
  n, t = g['v_x'].shape[:2]
  streams = oracle.legacy_streams(spec, g['seeds'], t)
  outs = {}
  for mf in ('1', '0'):
    monkeypatch.setenv('PBH_GIBBS_MFMA', mf)
    outs[mf], _ = _run_replay(spec, golden_init(name, n), streams, debug=False)
  assert np.array_equal(outs['1']['v_x'], outs['0']['v_x'])
  assert _rel_err(outs['1']['v_p'], outs['0']['v_p']) <= 1e-13
  assert _rel_err(outs['1']['v_p'], g['v_p']) <= RTOL


@pytest.mark.parametrize('n_obs', [7, 129, 1000, 20000])
def test_iid_normal_pairwise_tree_matches_numpy(n_obs):
  """PD.prod's np.sum over observations (pd.py:368) is reproduced by the
  kernel's numpy pairwise tree: leaf < 8, 8-accumulator leaves, the split
  recursion beyond 128 terms, and the global-memory path beyond the LDS
  stage (> 16 384 observations)."""
  g = oracle.load_golden('metrohast_norm1d')
  spec = oracle.golden_spec('metrohast_norm1d', g)
  spec['target']['obs'] = np.random.RandomState(n_obs).normal(50., 10., n_obs)
  n, t = 64, 40
  streams = oracle.legacy_streams(spec, np.arange(n) + 123, t)
  init = golden_init('metrohast_norm1d', n)
  out, _ = _run_replay(spec, init, streams, debug=True)
  ref = oracle.run_mh(spec, init, streams)
  assert np.array_equal(out['u'], ref['u'])
  assert _rel_err(out['p_p'], ref['p_p']) <= RTOL
  assert _rel_err(out['v_x'], ref['v_x'], 1.) <= RTOL


@pytest.mark.parametrize('name', ['metrohast_norm1d', 'gmm2'])
def test_production_modes_agree_with_reference_arithmetic(name):
  """Production Philox (fast densities, filtered acceptance incl. the
  e-tempered tuple-tran form of App. A-1) against PHILOX_F64 (libm fp64
  Box-Muller, the reference's arithmetic): the same law.  Both runs start
  from the same init, so every step's expectation is the same under the
  same law; the chains are independent, so the Monte-Carlo standard error of
  a post-burn-in average is the sd of the per-chain averages / sqrt(N) (it
  carries each chain's autocorrelation).  Means, second moments and the
  accept rate agree within 5 combined MCSE."""
  spec = oracle.golden_spec(name)
  n, t, burn = 4096, 800, 300
  res = {}
  for mode in ('philox', 'philox_f64'):
    eng = _engine(spec)
    eng.init_chains(golden_init(name, n))
    eng.set_rng(mode, seed=77 if mode == 'philox' else 78)
    eng.alloc_trace(t, 1)
    eng.run(t)
    tr = eng.trace()
    eng.close()
    v = tr['v_x'][:, burn:]                       # [N, T', d]
    u = tr['u'][:, burn:].astype(np.float64)[..., None]
    draws = {'mean': v, 'sq': v * v, 'acc': u}   # [N, T', d] per statistic
    res[mode] = {k: (a.mean(axis=1).mean(axis=0),
                     a.mean(axis=1).std(axis=0, ddof=1) / np.sqrt(n),
                     a.reshape(-1, a.shape[-1]).std(axis=0))
                 for k, a in draws.items()}
  for k in ('mean', 'sq', 'acc'):
    (m1, e1, _), (m0, e0, sd) = res['philox'][k], res['philox_f64'][k]
    z = np.abs(m1 - m0) / np.sqrt(e1 ** 2 + e0 ** 2)
    assert np.all(z < 5), (name, k, m1, m0, z)
    # the band is tight enough to mean something: the MCSE is under 5 % of
    # the statistic's own spread over the draws (a multimodal target's
    # coordinate mean can sit near 0, so |mean| is no scale)
    assert np.all(np.maximum(e1, e0) < 0.05 * sd), (name, k, e1, e0, sd)


@pytest.mark.parametrize('lanes', ['2', '4'])
def test_gmm_lane_pair_kernel_matches_one_lane_kernel(monkeypatch, lanes):
  """cfg5 form: the multi-lane GMM kernel (components dealt over 2 or 4
  lanes) draws the same Philox stream as the one-chain-per-lane kernel; its
  log-sum-exp differs only in rounding, so chains, accept bits and moments
  agree and log-densities agree to ~1e-14 (ragged chain count)."""
  from probayes_amd import Engine
  spec = oracle.golden_spec('gmm2')
  n, t = 3000, 300
  outs = {}
  monkeypatch.setenv('PBH_GMM_LANES', lanes)
  for no_pair in ('0', '1'):
    monkeypatch.setenv('PBH_NO_PAIR', no_pair)
    eng = Engine(spec)
    eng.init_chains(golden_init('gmm2', n))
    eng.set_rng('philox', seed=5)
    eng.alloc_trace(t, 1)
    eng.run(t, steps_per_launch=128)
    outs[no_pair] = (eng.trace(), eng.moments())
    eng.close()
  (tp, mp), (t1, m1) = outs['0'], outs['1']
  assert np.array_equal(tp['u'], t1['u'])
  np.testing.assert_allclose(tp['v_x'], t1['v_x'], rtol=0, atol=1e-12)
  assert _rel_err(tp['v_p'], t1['v_p']) <= 1e-13
  assert np.array_equal(mp['n_acc'], m1['n_acc'])
  np.testing.assert_allclose(mp['sum'], m1['sum'], rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize('spl', [64, 20])
@pytest.mark.parametrize('mom', [True, False])
def test_gmm_quad_steady_state_form_is_the_general_form(monkeypatch, mom, spl):
  """The quad kernel's steady-state launch (whole groups of 8 steps where
  the launch's start and length allow -- 64-step launches -- else of 4 --
  20-step launches; no per-step range / record tests, branch-free stores) is
  bit-for-bit the general form (PBH_GMM_FULL=0); ragged chain count,
  several launches."""
  from probayes_amd import Engine
  spec = oracle.golden_spec('gmm2')
  n, t = 3000 + 5, 200
  outs = {}
  for full in ('1', '0'):
    monkeypatch.setenv('PBH_GMM_FULL', full)
    eng = Engine(spec)
    eng.init_chains(golden_init('gmm2', n))
    eng.set_rng('philox', seed=9)
    eng.set_collect(moments=mom)
    eng.alloc_trace(t, 1)
    eng.run(t, steps_per_launch=spl)
    outs[full] = (eng.trace(), eng.moments() if mom else None, eng.state())
    eng.close()
  (ta, ma, sa), (tb, mb, sb) = outs['1'], outs['0']
  for k in ('v_x', 'v_p', 'u'):
    assert np.array_equal(ta[k], tb[k]), k
  assert np.array_equal(sa[0], sb[0]) and np.array_equal(sa[1], sb[1])
  if mom:
    for k in ('sum', 'sumsq', 'n_acc'):
      assert np.array_equal(ma[k], mb[k]), k


def test_gmm_quad_full_size_cfg5_is_the_general_form(monkeypatch):
  """cfg5's per-GPU share at full size -- 32 768 chains, an 8-step warm-up,
  then one 2 000-step launch (the steady-state form in 8-step groups) --
  equals the general form (PBH_GMM_FULL=0) bit for bit: the final state and
  the device reductions of the whole trace (per-chain sums, sums of
  squares and accept counts, and the recorded v.prob's expectation)."""
  from probayes_amd import Engine
  spec = oracle.golden_spec('gmm2')
  n, t = 32768, 2000
  outs = {}
  for full in ('1', '0'):
    monkeypatch.setenv('PBH_GMM_FULL', full)
    eng = Engine(spec)
    eng.init_chains(golden_init('gmm2', n))
    eng.set_rng('philox', seed=23)
    eng.set_collect(moments=False)
    eng.run(8)
    eng.alloc_trace(t, 1)
    eng.run(t)
    st = eng.trace_stats(0, t)
    ex = eng.trace_expectation(0, t)
    outs[full] = (eng.state(), st, ex)
    eng.close()
  (sa, ta, ea), (sb, tb, eb) = outs['1'], outs['0']
  assert np.array_equal(sa[0], sb[0]) and np.array_equal(sa[1], sb[1])
  for k in ('sum', 'sumsq', 'n_acc'):
    assert np.array_equal(ta[k], tb[k]), k
  assert np.array_equal(ea, eb)
  assert ta['n_acc'].min() > 0   # every chain moved


@pytest.mark.parametrize('pair', ['1', '0'])
@pytest.mark.parametrize('n', [4096 + 5, 37])
def test_iid_steady_state_form_is_the_general_form(monkeypatch, pair, n):
  """cfg1's steady-state launch (iid-Normal target, spherical delta, ufun on
  sigma, uniform prior, e-tempered ratio form) -- on one lane per chain
  (mh_iid_full_kernel, the default, PBH_IID_PAIR=0) or on lane pairs
  (mh_iid_pair_kernel, opt-in PBH_IID_PAIR=1, measured slower) -- is
  bit-for-bit mh_kernel's general form
  (PBH_IID_FULL=0): ragged chain counts (padding lanes write nothing; an odd
  number of 32-chain wavefronts leaves the last accept word half-owned),
  launches of 1 and 13 steps starting on either step of a pair, chains
  started outside the prior box (density -inf until they enter it)."""
  from probayes_amd import Engine
  spec = oracle.golden_spec('metrohast_norm1d')
  t = 61
  init = golden_init('metrohast_norm1d', n)
  init[::89, 1] = 30.   # sigma outside (5, 20)
  outs = {}
  monkeypatch.setenv('PBH_IID_PAIR', pair)
  for full in ('1', '0'):
    monkeypatch.setenv('PBH_IID_FULL', full)
    eng = Engine(spec)
    eng.init_chains(init)
    eng.set_rng('philox', seed=13)
    eng.alloc_trace(t, 1)
    eng.run(1)
    eng.run(4, steps_per_launch=1)
    eng.run(t - 5, steps_per_launch=13)
    outs[full] = (eng.trace(), eng.state())
    eng.close()
  (ta, sa), (tb, sb) = outs['1'], outs['0']
  for k in ('v_x', 'v_p', 'u'):
    assert np.array_equal(ta[k], tb[k]), k
  assert np.array_equal(sa[0], sb[0]) and np.array_equal(sa[1], sb[1])
  assert 0 < tb['u'].mean() < 1


@pytest.mark.parametrize('which', ['golden', 'bench'])
def test_pair_steady_state_form_is_the_general_form(monkeypatch, which):
  """The lane-pair kernel's steady-state launch (FULL: whole step pairs,
  branch-free stores, the next pair's draws pipelined beside the current
  pair's steps, the state's range bit carried as a mask) is bit-for-bit the
  general form (PBH_PAIR_FULL=0): launches starting and ending on either step
  of a pair, chains far in the tails (|lp| > 700: the exact decision), the
  golden diag10 spec (nonzero proposal loc) and the bench's cfg2 spec."""
  import bench
  from probayes_amd import Engine
  spec = oracle.golden_spec('diag10') if which == 'golden' else bench.cfg2_spec()
  # the bench spec at a chain count whose last 8-wave workgroup is partial
  n, t = (4096 if which == 'golden' else 4096 + 96), 61
  init = np.zeros((n, 10)) if which == 'bench' else golden_init('diag10', n)
  init[::97] += 40.   # log-density far below -700
  outs = {}
  for full in ('1', '0'):
    monkeypatch.setenv('PBH_PAIR_FULL', full)
    eng = Engine(spec)
    eng.init_chains(init)
    eng.set_rng('philox', seed=11)
    eng.alloc_trace(t, 1)
    eng.run(1)
    eng.run(4, steps_per_launch=1)
    eng.run(t - 5, steps_per_launch=13)
    outs[full] = (eng.trace(), eng.state())
    eng.close()
  (ta, sa), (tb, sb) = outs['1'], outs['0']
  for k in ('v_x', 'v_p', 'u'):
    assert np.array_equal(ta[k], tb[k]), k
  assert np.array_equal(sa[0], sb[0]) and np.array_equal(sa[1], sb[1])
  assert 0 < tb['u'].mean() < 1
  # past step 1 the far chains never move: both densities underflow the
  # ratio form's exp (rescale -> 0), so the exact decision rejects, as the
  # reference's sp_utils.py ratio does
  assert tb['u'][::97, 1:].max() == 0


@pytest.mark.parametrize('name,thin,spl', [('diag10', 3, 0), ('diag10', 4, 7),
                                           ('gmm2', 4, 9), ('gibbs8', 5, 13),
                                           ('gibbs_sweep2', 3, 5)])
def test_production_thinning_equals_every_kth_step(name, thin, spl):
  """Production kernels (lane-pair MH, GMM lane-pair, Gibbs): a thinned
  trace is exactly every thin-th record of the full trace, whatever the
  launch split (the RNG is keyed by absolute step)."""
  from probayes_amd import Engine
  spec = oracle.golden_spec(name)
  n, t = 200, 60

  def run(th, sp):
    eng = Engine(spec)
    eng.init_chains(golden_init(name, n))
    eng.set_rng('philox', seed=31)
    eng.alloc_trace(t // th, th)
    eng.run(t, steps_per_launch=sp)
    tr, mom = eng.trace(), eng.moments()
    eng.close()
    return tr, mom

  full, mf = run(1, 0)
  part, mp = run(thin, spl)
  for k in ('v_x', 'v_p', 'u'):
    np.testing.assert_array_equal(part[k], full[k][:, thin - 1::thin])
  np.testing.assert_array_equal(mp['n_acc'], mf['n_acc'])
  np.testing.assert_allclose(mp['sum'], mf['sum'], rtol=1e-13, atol=1e-12)


@pytest.mark.parametrize('name,n,t', [('gibbs8', 32768, 48), ('gmm2', 32768, 120)])
def test_full_size_cfg3_cfg5_replay_parity(name, n, t):
  """BASELINE cfg3 / cfg5 per-GPU widths in replay mode: 256 sampled chains
  match the oracle step for step; trace/moment invariants hold for all."""
  from probayes_amd.replay import legacy_streams_parallel
  spec = oracle.golden_spec(name)
  seeds = np.arange(n, dtype=np.int64) + 3_000_000
  streams = legacy_streams_parallel(spec, t, seeds, processes=16)
  init = golden_init(name, n)
  out, mom = _run_replay(spec, init, streams, debug=False)
  assert np.array_equal(mom['n_acc'], out['u'].sum(axis=1))
  np.testing.assert_allclose(mom['sum'], out['v_x'].sum(axis=1), rtol=1e-12,
                             atol=1e-9)
  pick = np.random.RandomState(9).choice(n, 256, replace=False)
  run = oracle.run_gibbs if spec['scores'] == 'gibbs' else oracle.run_mh
  ref = run(spec, init[pick], streams[:, :, pick])
  assert np.array_equal(out['u'][pick], ref['u'])
  assert _rel_err(out['v_x'][pick], ref['v_x'], 1.) <= RTOL
  assert _rel_err(out['v_p'][pick], ref['v_p']) <= RTOL


@pytest.mark.parametrize('d,n', [(32, 70), (16, 1), (12, 33), (3, 1)])
def test_extreme_dims_and_chain_counts_replay(d, n):
  """Largest compiled dimension (32: lane-pair kernel with 16 dims per half),
  a single chain, and ragged chain counts against the oracle."""
  from oracle.workloads import spec_diag10
  spec = spec_diag10({'mu': np.linspace(-1., 1., d),
                      'sigma': np.linspace(0.5, 2., d), 'step': 0.5})
  t = 40
  streams = oracle.legacy_streams(spec, np.arange(n) + 11, t)
  init = np.zeros((n, d))
  out, _ = _run_replay(spec, init, streams, debug=False)
  ref = oracle.run_mh(spec, init, streams)
  assert np.array_equal(out['u'], ref['u'])
  assert _rel_err(out['v_x'], ref['v_x'], 1.) <= RTOL
  assert _rel_err(out['v_p'], ref['v_p']) <= RTOL


@pytest.mark.parametrize('name,rng', [('diag10', 'philox'), ('gmm2', 'philox'),
                                      ('metrohast_norm1d', 'philox_f64'),
                                      # production ufun: the carried logs
                                      ('metrohast_norm1d', 'philox'),
                                      ('metrohast_norm1d', 'xoshiro'),
                                      ('diag10', 'xoshiro'),
                                      ('gibbs8', 'philox')])
def test_checkpoint_resume_continues_the_run(name, rng):
  """pbh_get_checkpoint / pbh_restore: a fresh engine restored
  from a checkpoint at step 40 continues the uninterrupted run step for step
  (production Gibbs: states exact, v.prob to the O(d) refresh tolerance)."""
  from probayes_amd import Engine
  spec = oracle.golden_spec(name)
  n, t, t1 = 1000 + 7, 100, 40

  def engine():
    e = Engine(spec)
    e.init_chains(golden_init(name, n))
    e.set_rng(rng, seed=21)
    return e
  full = engine()
  full.alloc_trace(t, 1)
  full.run(t, steps_per_launch=16)
  ref = full.trace()
  full.close()
  a = engine()
  a.run(t1, steps_per_launch=16)
  ck = a.checkpoint()
  a.close()
  assert ck['step'] == t1 and ck['has_pred']
  b = engine()
  b.restore(ck)
  b.alloc_trace(t - t1, 1)
  b.run(t - t1, steps_per_launch=16)
  got = b.trace()
  b.close()
  assert np.array_equal(got['v_x'], ref['v_x'][:, t1:])
  assert np.array_equal(got['u'], ref['u'][:, t1:])
  if spec['scores'] == 'gibbs':
    assert _rel_err(got['v_p'], ref['v_p'][:, t1:]) <= 1e-9
  else:
    assert np.array_equal(got['v_p'], ref['v_p'][:, t1:])


def test_checkpoint_with_device_legacy_streams_and_shape_checks():
  """The legacy-stream part of a checkpoint (MT19937 key, position, cached
  gauss): a fresh engine seeded the same way and restored continues the
  uninterrupted reference-identical run; a checkpoint whose legacy state does
  not match the engine's layout or chain count is refused before any copy
  (the C side copies words x N values from the arrays)."""
  from probayes_amd import Engine
  name = 'diag10'
  spec = oracle.golden_spec(name)
  n, t, t1 = 300, 30, 11
  seeds = 1000 + np.arange(n)

  def engine():
    e = Engine(spec)
    e.init_chains(golden_init(name, n))
    e.set_rng('replay')
    e.seed_legacy(seeds)
    return e
  full = engine()
  full.legacy_replay(t)
  full.alloc_trace(t, 1)
  full.run(t)
  ref = full.trace()
  full.close()
  a = engine()
  a.legacy_replay(t1)
  a.run(t1)
  ck = a.checkpoint()
  a.close()
  assert ck['mt'] is not None
  b = engine()
  for bad in ({'key': ck['mt']['key'][:624]}, {'pos': ck['mt']['pos'][:-1]},
              {'gauss': np.zeros(n + 1)}):
    with pytest.raises(ValueError, match='legacy state'):
      b.restore(dict(ck, mt=dict(ck['mt'], **bad)))
  with pytest.raises(ValueError, match='xoshiro'):
    b.restore(dict(ck, xo=np.zeros(5, np.uint32)))
  b.restore(ck)
  b.legacy_replay(t - t1)
  b.alloc_trace(t - t1, 1)
  b.run(t - t1)
  got = b.trace()
  b.close()
  assert np.array_equal(got['u'], ref['u'][:, t1:])
  assert np.array_equal(got['v_x'], ref['v_x'][:, t1:])
