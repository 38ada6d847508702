"""User-conditional Gibbs (examples/mcmc/gibbs_linreg.py): the oracle against
the reference's recorded chains, the descriptor conditional, the C-ABI's
argument errors (CPU), and the HIP kernel against the oracle (GPU)."""
import numpy as np
import pytest

from oracle.linreg import linreg_streams, run_linreg, HYPER, VSETS
from probayes_amd import _lib, linreg

GOLDEN = 'tests/golden/gibbs_linreg.npz'


def _golden(root):
  import os
  g = np.load(os.path.join(root, GOLDEN))
  n = len(g['seeds'])
  return g, g['param_x_obs'], g['param_y_obs'], np.tile(g['param_init'], (n, 1))


def test_oracle_matches_reference_bitwise(root):
  """tools/gen_golden.py recorded the reference's SP chains (rf.py:413-462
  calling cond_reg; fresh SP per chain, np.random.seed(seed))."""
  g, x, y, init = _golden(root)
  t = g['v_x'].shape[1]
  o = run_linreg(x, y, init, linreg_streams(g['seeds'], t, len(x)))
  assert np.array_equal(o['v_x'], g['v_x'])
  assert np.array_equal(o['v_p'], g['v_p'])
  assert np.all(g['u'] == 1)            # gibbs: every step accepted
  assert np.array_equal(g['p_x'], g['v_x'])


def test_descriptor_conditional_draws_like_cond_reg(root):
  """LinRegConditional in the reference's calling convention (one unknown per
  call, NumPy's global stream) gives the golden chain."""
  g, x, y, init = _golden(root)
  cond = linreg.LinRegConditional(len(x))
  for c in range(2):
    np.random.seed(int(g['seeds'][c]))
    vals = dict(zip(linreg.KEYS, init[c]))
    for t in range(g['v_x'].shape[1]):
      key = linreg.KEYS[t % 3]
      vals[key] = cond(x, y, unknown=key, **vals)
      assert [vals[k] for k in linreg.KEYS] == list(g['v_x'][c, t])


def test_abi_rejects_bad_arguments():
  x = np.zeros(4)
  init = np.ones((2, 3))
  with pytest.raises(ValueError):
    linreg.run(x, np.zeros(5), init, 3)
  with pytest.raises(_lib.PbhError):    # n_obs above the LDS cap
    linreg.run(np.zeros(10000), np.zeros(10000), init, 3)
  with pytest.raises(ValueError):       # replay needs [T, N] draws
    linreg.run(x, x, init, 3, rng='replay', rand=np.zeros((2, 2)))
  with pytest.raises(_lib.PbhError):
    linreg.run(x, x, init, 3, hyper=(0., 0., 0., 1., 1., 1.))


def _data(n_obs, seed=5):
  rs = np.random.RandomState(seed)
  x = rs.normal(0, 1, size=n_obs)
  return x, rs.normal(1.5 * x - 1., 0.5)


@pytest.mark.gpu
def test_replay_reproduces_reference_chains(root):
  g, x, y, init = _golden(root)
  t = g['v_x'].shape[1]
  st = linreg_streams(g['seeds'], t, len(x))
  out = linreg.run(x, y, init, t, rng='replay', rand=st)
  rel = np.abs(out['v_x'] - g['v_x']) / np.maximum(np.abs(g['v_x']), 1.)
  assert rel.max() <= 1e-12, rel.max()
  assert np.max(np.abs(out['v_p'] - g['v_p']) / np.abs(g['v_p'])) <= 1e-12
  assert np.array_equal(out['final_x'], out['v_x'][:, -1])


@pytest.mark.gpu
@pytest.mark.parametrize('n_obs', [1, 7, 60, 129, 1000, 8192])
def test_replay_matches_oracle_ragged(n_obs):
  """Edge sizes of the pairwise sums (n < 8, leaf, split tree, LDS cap) and
  a ragged chain count."""
  x, y = _data(n_obs)
  n, t = 77, 40
  init = np.column_stack([np.full(n, -0.5), np.full(n, 1.0),
                          np.linspace(0.3, 2., n)])
  st = linreg_streams(np.arange(100, 100 + n), t, n_obs)
  ref = run_linreg(x, y, init, st)
  out = linreg.run(x, y, init, t, rng='replay', rand=st)
  rel = np.abs(out['v_x'] - ref['v_x']) / np.maximum(np.abs(ref['v_x']), 1.)
  assert rel.max() <= 1e-12, rel.max()
  relp = np.abs(out['v_p'] - ref['v_p']) / np.maximum(np.abs(ref['v_p']), 1.)
  assert relp.max() <= 1e-12, relp.max()


@pytest.mark.gpu
def test_fast_form_matches_reference_arithmetic_on_the_same_draws():
  """PHILOX (sufficient statistics) and PHILOX_F64 (reference arithmetic)
  read the same Philox draws: the chains agree to rounding."""
  x, y = _data(60)
  n, t = 4096, 300
  init = np.tile([-0.9, 1.4, 0.6], (n, 1))
  a = linreg.run(x, y, init, t, rng='philox', seed=11)
  b = linreg.run(x, y, init, t, rng='philox_f64', seed=11)
  assert np.max(np.abs(a['v_x'] - b['v_x'])) <= 1e-9
  assert np.max(np.abs(a['v_p'] - b['v_p']) / np.abs(b['v_p'])) <= 1e-9


@pytest.mark.gpu
def test_sharding_and_launch_split_invariance():
  x, y = _data(60)
  n, t = 1000, 60
  init = np.tile([-0.9, 1.4, 0.6], (n, 1))
  full = linreg.run(x, y, init, t, rng='philox', seed=3)
  lo = linreg.run(x, y, init[:400], t, rng='philox', seed=3)
  hi = linreg.run(x, y, init[400:], t, rng='philox', seed=3, chain_offset=400)
  assert np.array_equal(np.concatenate([lo['v_x'], hi['v_x']]), full['v_x'])
  first = linreg.run(x, y, init, 25, rng='philox', seed=3)
  second = linreg.run(x, y, first['final_x'], t - 25, rng='philox', seed=3,
                      step0=25)
  assert np.array_equal(second['v_x'], full['v_x'][:, 25:])


@pytest.mark.gpu
def test_posterior_matches_oracle_within_monte_carlo_error():
  """Posterior means and sds of (beta_0, beta_1, y_sigma) from Philox chains
  against the oracle's NumPy-stream chains (the reference's law)."""
  x, y = _data(60, seed=9)
  burn, t = 30, 150
  n_gpu, n_cpu = 16384, 2048
  init = np.tile([0., 0., 1.], (n_gpu, 1))
  g = linreg.run(x, y, init, t, rng='philox', seed=21)['v_x'][:, burn:]
  r = run_linreg(x, y, init[:n_cpu], linreg_streams(
      np.arange(5000, 5000 + n_cpu), t, len(x)))['v_x'][:, burn:]
  for k in range(3):
    gm, rm = g[:, -1, k].mean(), r[:, -1, k].mean()
    sd = r[:, -1, k].std()
    assert abs(gm - rm) <= 5 * sd * np.sqrt(1 / n_gpu + 1 / n_cpu), (k, gm, rm)
    assert abs(g[:, -1, k].std() / sd - 1) <= 0.1, k


def _facade(root, cond=None):
  import probayes_amd as pb
  from mcmc_examples import TFUN_WORKLOADS
  builder, params, n, t, seed0 = TFUN_WORKLOADS['gibbs_linreg']
  g, x, y, _ = _golden(root)
  params = dict(params, x_obs=x, y_obs=y)
  if cond is not None:
    params['cond'] = cond
  return builder(pb, params) + (g, t)


def test_facade_lowers_the_descriptor_and_refuses_other_tfuns(root):
  import probayes_amd as pb
  process, init, extra, kwds, keys, g, t = _facade(root, linreg.LinRegConditional)
  spec = process.lower(extra, iid=True, joint=True)
  assert spec['kind'] == 'linreg' and spec['names'] == list(linreg.KEYS)
  assert spec['vsets'] == [(-6., 6.), (-6., 6.), (0.001, 10.)]
  assert process.lower(extra, iid=True, joint=False)['vsets'] is None
  # the example's own closure cond_reg: identified by probing
  process2, _, extra2, _, _, _, _ = _facade(root)
  spec2 = process2.lower(extra2, iid=True, joint=True)
  assert spec2['kind'] == 'linreg' and spec2['hyper'] == (0., 1., 0., 1., 1., 1.)
  from mcmc_examples import linreg_cond
  x, y = spec2['x_obs'], spec2['y_obs']

  def wrong_scale(x, y, beta_0, beta_1, y_sigma, unknown):
    if unknown == 'beta_1':      # variance passed where NumPy wants the sd
      y_prec = 1 / y_sigma ** 2
      cond_var = 1 / (1. + y_prec * np.sum(x ** 2))
      return np.random.normal(cond_var * y_prec * np.sum(x * (y - beta_0)),
                              cond_var)
    return linreg_cond(x, y)(x, y, beta_0, beta_1, y_sigma, unknown)

  def two_draws(x, y, beta_0, beta_1, y_sigma, unknown):
    np.random.normal()
    return linreg_cond(x, y)(x, y, beta_0, beta_1, y_sigma, unknown)

  def other_hyper(x, y, beta_0, beta_1, y_sigma, unknown):
    return linreg_cond(x, y)(x, y, beta_0, beta_1, y_sigma, unknown,
                             beta_0_mu=0.25, y_sigma_beta=2.)
  for fn in (wrong_scale, two_draws):
    with pytest.raises(pb.NotLowerable):
      linreg.identify_conditional(fn, x, y)
  assert linreg.identify_conditional(other_hyper, x, y) == \
      (0.25, 1., 0., 1., 1., 2.)
  process.set_prob(lambda x, y, beta_0, beta_1, y_sigma: -(y - beta_0) ** 2,
                   pscale='log')
  with pytest.raises(pb.NotLowerable):
    process.lower(extra, iid=True, joint=True)


@pytest.mark.gpu
def test_example_script_reproduces_reference_chain(root):
  """np.random.seed(s); sampler; walk; SP(samples) as gibbs_linreg.py:74-78
  does, on NumPy's global stream."""
  for c in range(2):
    process, init, extra, kwds, keys, g, t = _facade(root)   # own cond_reg
    seed = int(g['seeds'][c])
    np.random.seed(seed)
    samples = process.walk(process.sampler(init, extra, stop=t, **kwds))
    summary = process(samples)
    for i, k in enumerate(keys):
      got = np.asarray(summary.v[k])
      assert np.max(np.abs(got - g['v_x'][c, :, i]) /
                    np.maximum(np.abs(g['v_x'][c, :, i]), 1.)) <= 1e-12
    assert np.max(np.abs(np.asarray(summary.v.prob) - g['v_p'][c]) /
                  np.abs(g['v_p'][c])) <= 1e-12
    assert summary.u.count(True) == t
    rs = np.random.RandomState(seed)
    for s in range(t):
      rs.standard_gamma(31.) if s % 3 == 2 else rs.standard_normal()
    assert np.random.random_sample() == rs.random_sample()


@pytest.mark.gpu
def test_batched_sampler_reproduces_all_reference_chains(root):
  process, init, extra, kwds, keys, g, t = _facade(root)   # own cond_reg
  n = len(g['seeds'])
  sm = process.sampler(init, extra, stop=t, chains=n, seeds=g['seeds'], **kwds)
  summary = process(process.walk(sm))
  for i, k in enumerate(keys):
    got = np.asarray(summary.v[k]).T          # [T, N] -> [N, T]
    assert np.max(np.abs(got - g['v_x'][:, :, i]) /
                  np.maximum(np.abs(g['v_x'][:, :, i]), 1.)) <= 1e-12
  sm = process.sampler(init, extra, stop=t, chains=4096, **kwds)   # philox
  summary = process(process.walk(sm))
  assert np.asarray(summary.v['y_sigma']).shape == (t, 4096)
  assert np.all(np.isfinite(np.asarray(summary.v.prob)))


@pytest.mark.gpu
@pytest.mark.parametrize('alpha', [31., 2.5, 1., 0.4])
def test_device_gamma_equals_numpy_randomstate(alpha):
  """pbh_legacy_draws: per chain NumPy's
  RandomState(seed) drawing gibbs_linreg's cond_reg order -- standard_gamma
  (alpha) on every third step, the legacy gauss otherwise -- on the device:
  the same draws (NumPy's legacy_standard_gamma: Marsaglia-Tsang over the
  polar gauss, the shape < 1 branch, shape 1 the exponential) and the same
  generator state after them, across calls.  The device logs are within an
  ulp of libm's, so the values agree to ~1e-15 relative and mostly exactly."""
  from probayes_amd import Engine
  from probayes_amd.spec import make_spec
  n = 200
  seeds = np.concatenate([[0, 1, 2 ** 32 - 1], np.arange(7, 7 + n - 3)])
  eng = Engine(make_spec(1, target={'kind': 'diag_gauss', 'mu': np.zeros(1),
                                    'sigma': np.ones(1)},
                         proposal={'kind': 'gauss', 'loc': 0., 'scale': 1.},
                         scores='hastings', pscale='log',
                         tran={'kind': 'const', 'value': 1.0, 'sym': True}))
  eng.init_chains(np.zeros((n, 1)))
  eng.seed_legacy(seeds)
  a = eng.legacy_draws(17, 0, 'linreg', alpha)
  b = eng.legacy_draws(40, 17, 'linreg', alpha)
  eng.close()
  dev = np.concatenate([a, b])
  ref = np.empty_like(dev)
  for c, sd in enumerate(seeds):
    rs = np.random.RandomState(int(sd))
    for t in range(dev.shape[0]):
      ref[t, c] = rs.standard_gamma(alpha) if t % 3 == 2 else rs.standard_normal()
  rel = np.abs(dev - ref) / np.maximum(np.abs(ref), 1e-300)
  assert rel.max() <= 4e-15, rel.max()
  # exact for most; shape < 1 goes through pow (the device's within ~1 ulp
  # of libm's)
  assert np.mean(dev == ref) > (0.95 if alpha >= 1. else 0.8)


@pytest.mark.gpu
def test_batched_sampler_at_full_width_on_device_streams(root):
  """The seeded linreg sampler at 65 536 chains: its RandomStates are drawn
  on the device (no per-chain Python loop); the golden chains, placed among
  the others, reproduce the reference's recorded chains."""
  process, init, extra, kwds, keys, g, t = _facade(root)
  n = 65536
  seeds = np.arange(n, dtype=np.int64) + 10 ** 6
  at = np.array([5, 40000, 65535])[:len(g['seeds'])]
  seeds[at] = g['seeds'][:len(at)]
  sm = process.sampler(init, extra, stop=t, chains=n, seeds=seeds, **kwds)
  summary = process(process.walk(sm))
  for i, k in enumerate(keys):
    got = np.asarray(summary.v[k]).T[at]      # [T, N] -> [N, T]
    want = g['v_x'][:len(at), :, i]
    assert np.max(np.abs(got - want) / np.maximum(np.abs(want), 1.)) <= 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize('vsets', [None, ((-1., -0.95), (1.3, 1.6), (0.4, 0.62))])
def test_replay_priors_and_vset_bounds_match_oracle(vsets):
  """joint=False (no prior) and tight vsets the chains leave: the
  NEARLY_NEGATIVE_INF terms of uniform_prob (rv_utils.py:30-38)."""
  x, y = _data(60)
  n, t = 130, 60
  init = np.tile([-0.98, 1.45, 0.5], (n, 1))
  st = linreg_streams(np.arange(300, 300 + n), t, 60)
  ref = run_linreg(x, y, init, st, vsets=vsets)
  out = linreg.run(x, y, init, t, rng='replay', rand=st, vsets=vsets)
  rel = np.abs(out['v_x'] - ref['v_x']) / np.maximum(np.abs(ref['v_x']), 1.)
  assert rel.max() <= 1e-12
  fin = np.isfinite(ref['v_p'])
  assert np.array_equal(fin, np.isfinite(out['v_p']))
  assert np.array_equal(ref['v_p'][~fin], out['v_p'][~fin])
  big = np.abs(ref['v_p']) > 1e300
  assert np.array_equal(big, np.abs(out['v_p']) > 1e300)
  if vsets is not None:
    assert big.any() and not big.all()
  ok = fin & ~big
  assert np.max(np.abs(out['v_p'][ok] - ref['v_p'][ok]) /
                np.abs(ref['v_p'][ok])) <= 1e-12


@pytest.mark.gpu
def test_lane_pair_kernel_equals_one_lane_kernel(monkeypatch):
  """PBH_LINREG_PAIR=1 runs linreg_pair_kernel (one chain per lane pair);
  the default PHILOX path runs the one-lane kernel.  Same draws and arithmetic: identical chains,
  including a ragged chain count and a launch starting mid-cycle."""
  x, y = _data(60)
  n, t = 1000 + 13, 77
  init = np.tile([-0.9, 1.4, 0.6], (n, 1))
  for step0 in (0, 1, 2):
    a = linreg.run(x, y, init, t, rng='philox', seed=8, step0=step0)
    monkeypatch.setenv('PBH_LINREG_PAIR', '1')
    b = linreg.run(x, y, init, t, rng='philox', seed=8, step0=step0)
    monkeypatch.delenv('PBH_LINREG_PAIR')
    assert np.array_equal(a['v_x'], b['v_x'])
    assert np.array_equal(a['v_p'], b['v_p'])
    assert np.array_equal(a['final_x'], b['final_x'])
    assert np.array_equal(a['final_p'], b['final_p'])


@pytest.mark.gpu
def test_consecutive_samplers_continue_the_cycle(root):
  """Three samplers on one process (gibbs_linreg_seg, recorded from the
  reference): each continues the paras RF's __cond_mod (rf.py:446-452) and
  NumPy's global stream."""
  import os
  import probayes_amd as pb
  from mcmc_examples import TFUN_WORKLOADS
  g = np.load(os.path.join(root, 'tests/golden/gibbs_linreg_seg.npz'))
  builder, params = TFUN_WORKLOADS['gibbs_linreg'][:2]
  for c in range(len(g['seeds'])):
    process, init, extra, kwds, keys = builder(pb, params)
    np.random.seed(int(g['seeds'][c]))
    got = []
    for stop in g['segments']:
      s = process(process.walk(process.sampler(init, extra, stop=int(stop),
                                               **kwds)))
      got.append(np.stack([np.asarray(s.v[k]) for k in keys], -1))
    got = np.concatenate(got)
    assert np.max(np.abs(got - g['v_x'][c]) /
                  np.maximum(np.abs(g['v_x'][c]), 1.)) <= 1e-12


@pytest.mark.gpu
def test_fast_form_is_stable_at_large_offsets():
  """The PHILOX form's centred sufficient statistics (x, y offset by 1e3):
  same chains as the reference arithmetic of PHILOX_F64 on the same draws."""
  rs = np.random.RandomState(2)
  x = 1000. + rs.normal(0, 1, 60)
  y = 2. + 0.004 * x + rs.normal(0, 0.5, 60)
  n, t = 2048, 120
  init = np.tile([2.0, 0.004, 0.5], (n, 1))
  a = linreg.run(x, y, init, t, rng='philox', seed=4, vsets=None)
  b = linreg.run(x, y, init, t, rng='philox_f64', seed=4, vsets=None)
  rel = np.abs(a['v_x'] - b['v_x']) / np.maximum(np.abs(b['v_x']), 1.)
  assert rel.max() <= 1e-9, rel.max()
  assert np.max(np.abs(a['v_p'] - b['v_p']) / np.abs(b['v_p'])) <= 1e-9
