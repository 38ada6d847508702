"""The SP facade: the examples/mcmc scripts written against probayes_amd.

CPU tests: every example lowers to exactly the workload spec the oracle was
pinned with.  GPU tests: the example scripts run end to end on the engine and
reproduce the reference's recorded chains -- one chain per sampler drawing
from NumPy's GLOBAL legacy stream after np.random.seed (the reference's own
convention), and all chains at once with chains=N, seeds=[...].
"""
import numpy as np
import pytest

import oracle
import probayes_amd as pb
from mcmc_examples import WORKLOADS as _W, DELTA_WORKLOADS

WORKLOADS = dict(_W, **DELTA_WORKLOADS)


def _spec_equal(a, b, path=''):
  bad = []
  if isinstance(a, dict):
    if set(a) != set(b):
      return [path + ':keys']
    for k in a:
      bad += _spec_equal(a[k], b[k], path + '.' + k)
  elif isinstance(a, (np.ndarray, list, tuple)):
    if not np.array_equal(np.asarray(a), np.asarray(b)):
      bad.append(path)
  elif a != b:
    bad.append(path)
  return bad


def _build(name):
  builder, params, n, t, seed0 = WORKLOADS[name]
  g = oracle.load_golden(name)
  params = oracle.workloads.golden_params(g) if params else params
  process, init, extra, kwds, keys = builder(pb, params)
  return process, init, extra, kwds, keys, g


@pytest.mark.parametrize('name', sorted(WORKLOADS))
def test_examples_lower_to_the_oracle_spec(name):
  process, init, extra, kwds, keys, g = _build(name)
  spec = process.lower(extra, kwds.get('iid', False), kwds.get('joint', False))
  ref = oracle.golden_spec(name, g)
  for k in ('dim', 'pscale', 'scores', 'ufun', 'target', 'proposal', 'tran',
            'prior'):
    if spec['scores'] == 'gibbs' and k == 'tran':
      continue
    assert not _spec_equal(spec[k], ref[k]), (k, _spec_equal(spec[k], ref[k]))


def test_unrecognised_forms_fail_loudly():
  import scipy.stats
  x = pb.RV('x', vtype=float, vset=(-np.inf, np.inf))
  process = pb.SP(x)
  process.set_prob(lambda **kw: np.cos(kw['x']))
  process.set_tran(lambda **kw: 1.)
  process.set_delta(lambda: process.Delta(x=scipy.stats.norm.rvs()))
  process.set_scores('hastings')
  with pytest.raises(pb.NotLowerable):
    process.lower()
  process.set_prob(scipy.stats.norm.pdf, order={'x': 0})
  process.set_delta(lambda: process.Delta(x=np.random.uniform()))
  with pytest.raises(pb.NotLowerable):
    process.lower()


def _golden_rtol(a, b):
  den = np.maximum(np.abs(b), 1.)
  return float(np.max(np.abs(a - b) / den))


@pytest.mark.gpu
@pytest.mark.parametrize('name', sorted(WORKLOADS))
def test_example_scripts_reproduce_reference_chains(name):
  """np.random.seed(s); build; sampler; walk; SP(samples) -- as the reference
  example scripts do -- gives the reference's recorded chain."""
  builder, params, n, t, seed0 = WORKLOADS[name]
  g = oracle.load_golden(name)
  for c in range(2):
    process, init, extra, kwds, keys, _ = _build(name)
    np.random.seed(int(g['seeds'][c]))
    args = (init,) if extra is None else (init, extra)
    sampler = process.sampler(*args, stop=t, **kwds)
    samples = process.walk(sampler)
    summary = process(samples)
    for i, k in enumerate(keys):
      assert _golden_rtol(np.asarray(summary.v[k]), g['v_x'][c, :, i]) <= 1e-12
    assert _golden_rtol(np.asarray(summary.v.prob), g['v_p'][c]) <= 1e-12
    assert summary.u.count(True) == int(g['u'][c].sum())
    # the global legacy stream advanced exactly as the reference's did
    spec = oracle.golden_spec(name, g)
    states = []
    oracle.legacy_streams(spec, g['seeds'][c:c + 1], t, states=states)
    assert np.random.random_sample() == states[0].random_sample()


@pytest.mark.gpu
@pytest.mark.parametrize('name', ['metrohast_norm1d', 'diag10', 'gibbs8',
                                  'gmm2', 'mcmc_prob6', 'bound_sphere2',
                                  'bound_list3', 'pervar3', 'randint2'])
def test_batched_sampler_reproduces_all_reference_chains(name):
  builder, params, n, t, seed0 = WORKLOADS[name]
  process, init, extra, kwds, keys, g = _build(name)
  args = (init,) if extra is None else (init, extra)
  sampler = process.sampler(*args, stop=t, chains=n, seeds=g['seeds'], **kwds)
  summary = process(process.walk(sampler))
  for i, k in enumerate(keys):
    got = np.asarray(summary.v[k]).T            # [N, T]
    assert _golden_rtol(got, g['v_x'][:, :, i]) <= 1e-12
  assert summary.u.count(True) == int(g['u'].sum())
  if sampler.spec['proposal']['kind'] != 'gibbs':
    # the thresholds t (sp.py:249): kept by the fused kernel
    # (pbh_set_record_threshold), each chain's RandomState's last draw of
    # the step, bit for bit
    import oracle
    ref = oracle.legacy_streams(sampler.spec, g['seeds'], t)[:, -1, :]
    np.testing.assert_array_equal(np.asarray(summary.t), ref)


@pytest.mark.gpu
@pytest.mark.parametrize('rng', ['philox', 'xoshiro'])
def test_batched_philox_sampler_posterior(rng):
  """metrohast_norm1d posterior with 4096 production chains."""
  process, init, extra, kwds, keys, g = _build('metrohast_norm1d')
  sampler = process.sampler(init, extra, stop=2000, chains=4096, rng=rng,
                            seed=7, **kwds)
  summary = process(process.walk(sampler))
  mus = np.asarray(summary.v['mu'])[500:]
  sig = np.asarray(summary.v['sigma'])[500:]
  x = g['param_x_obs']
  assert abs(np.mean(mus) - np.mean(x)) < 0.5
  assert abs(np.median(sig) - np.std(x)) < 1.5


def test_covariance_tran_routes_like_the_reference():
  """rf.py:210-220 (cholesky tfun), dependence.py:316-326 (subfield names),
  sd.py:97-105 (SP.set_tran(ndarray) fails in leafs_roots)."""
  cov = np.array([[1.5, -1.0], [-1.0, 2.]])
  x = pb.RV('x', vtype=float, vset=(-10., 10.))
  y = pb.RV('y', vtype=float, vset=(-10., 10.))
  xy = x & y
  xy.set_tran(cov)
  np.testing.assert_array_equal(xy.lud, np.linalg.cholesky(cov))
  process = pb.SP(xy)
  with pytest.raises(ValueError):
    process.set_tran(cov)
  with pytest.raises(AssertionError):
    process.set_tran('roots')              # a one-field SP has only 'leafs'
  with pytest.raises(AssertionError):
    xy.set_tran(np.eye(3))
  with pytest.raises(AssertionError):
    xy.set_tfun(np.array([[1., 2.], [3., 4.]]))   # not triangular
  xy.set_delta([0.5])
  import scipy.stats
  def lp(**kw):
    return scipy.stats.norm.logpdf(kw['x'], 0., 1.) + \
        scipy.stats.norm.logpdf(kw['y'], 0., 2.)
  process.set_prob(lp, pscale='log')
  process.set_tran('leafs')
  process.set_delta('leafs')
  process.set_scores('hastings')
  spec = process.lower()
  np.testing.assert_array_equal(spec['proposal']['tfun'], np.linalg.cholesky(cov))
  assert spec['proposal']['kind'] == 'uniform'
  assert spec['tran'] == {'kind': 'const', 'value': 1.0, 'sym': False}


@pytest.mark.gpu
def test_summary_conditionalise_fails_as_reference():
  """SP(samples, conditionalise=True) (sp.py:132-149, 196-197) raises
  TypeError on an MH summary in the reference (tests/golden/pd_ops.npz
  meta cond_errors); the facade raises the same."""
  builder, params, n, t, seed0 = WORKLOADS['diag10']
  process, init, extra, kwds, keys, g = _build('diag10')
  np.random.seed(int(g['seeds'][0]))
  args = (init,) if extra is None else (init, extra)
  samples = process.walk(process.sampler(*args, stop=8, **kwds))
  assert process(samples).v is not None
  with pytest.raises(TypeError):
    process(samples, conditionalise=True)


def test_delta_forms_lower_and_fail_like_the_reference():
  """field.py:220-317 / variable.py:376-410 argument handling: the
  reference's assertion and construction errors, and NotLowerable for the
  forms without a kernel."""
  x = pb.RV('x', vtype=float, vset=[-1., 1.])
  y = pb.RV('y', vtype=float, vset=(-np.inf, np.inf))
  n = pb.RV('n', vtype=int, vset=range(5))
  assert (x.lo_incl, x.hi_incl, y.lo_incl, y.hi_incl) == (True, True, False, False)
  assert n.length == 5 and list(n.vlims) == [0., 4.]
  r = pb.RV('r', vtype=float, vset=[(3.,), 1.])    # re-ordered limits
  assert list(r.vlims) == [1., 3.] and r.lo_incl and not r.hi_incl

  def proc(*rvs):
    p = pb.SP(pb.RF(*rvs))
    keys = [v.name for v in rvs]
    p.set_prob(lambda **kw: sum(__import__('scipy').stats.norm.logpdf(kw[k])
                                for k in keys), pscale='log')
    p.set_tran(lambda **kw: 1.)
    p.set_scores('hastings')
    return p

  p = proc(x, y)
  p.set_delta((0.1,), scale=True)
  with pytest.raises(AssertionError):     # y has infinite length
    p.lower()
  p.set_delta([0.1], scale=True)
  with pytest.raises(AssertionError):
    p.lower()
  p.set_delta([0.1], {'y': 0.3}, scale=True, bound=True)
  prop = p.lower()['proposal']
  assert prop['kind'] == 'uniform' and list(prop['delta']) == [0.2, 0.3]
  assert list(prop['bound']['xlo']) == [0, 1]
  p.set_delta((0.1,), {'y': 0.3})
  with pytest.raises(TypeError):
    p.lower()
  p.set_delta(p.Delta(x=(0.1,), y=None), bound=True)
  prop = p.lower()['proposal']
  assert list(prop['mode']) == [1, 0] and list(prop['bound']['on']) == [1, 0]
  p.set_delta(p.Delta(x=lambda: 0.1, y=[0.2]))
  with pytest.raises(pb.NotLowerable):
    p.lower()
  q = proc(n, x)
  q.set_delta(q.Delta(n=[0.5], x=[0.1]))
  with pytest.raises(ValueError):         # randint(0, 0)
    q.lower()
  q.set_delta([2], scale=False)
  prop = q.lower()['proposal']
  assert prop['kind'] == 'vardelta' and list(prop['mode']) == [3, 2]
  assert list(prop['vint']) == [1, 0]
  with pytest.raises(pb.NotLowerable):    # uniform prior over an int vset
    q.lower(joint=True)
  q.set_delta(lambda: q.Delta(n=1, x=0.), bound=True)
  with pytest.raises(pb.NotLowerable):
    q.lower()


@pytest.mark.gpu
def test_consecutive_samplers_continue_the_cycle():
  """Two samplers on one process, as tools/gen_golden.py ran the reference
  (gibbs_norm2d_seg): the second starts at the RF's CondCov phase
  (rf.py:446-452) on NumPy's continuing global stream."""
  from mcmc_examples import SEGMENTED
  base, segs, n = SEGMENTED['gibbs_norm2d_seg']
  g = oracle.load_golden('gibbs_norm2d_seg')
  builder, params = _W[base][:2]
  for c in range(n):
    process, init, extra, kwds, keys = builder(pb, params)
    np.random.seed(int(g['seeds'][c]))
    got = []
    for stop in segs:
      summary = process(process.walk(process.sampler(init, stop=stop, **kwds)))
      got.append(np.stack([np.asarray(summary.v[k]) for k in keys], -1))
    assert _golden_rtol(np.concatenate(got), g['v_x'][c]) <= 1e-12


def test_mixture_densities_trace_or_fail_loudly():
  """The H5 mixture written with NumPy (gmm2's own logp) lowers to the gmm
  form; scipy.special.logsumexp is the same form; anything else is
  NotLowerable."""
  import scipy.special
  import scipy.stats
  x = pb.RV('x', vtype=float, vset=(-np.inf, np.inf))
  y = pb.RV('y', vtype=float, vset=(-np.inf, np.inf))
  process = pb.SP(x & y)
  process.set_tran(lambda **kw: 1.)
  process.set_delta(lambda: process.Delta(x=scipy.stats.norm.rvs(scale=.5),
                                          y=scipy.stats.norm.rvs(scale=.5)))
  process.set_scores('hastings')
  logw, mu, sd = np.log([0.4, 0.6]), np.array([[0., 1.], [2., -1.]]), \
      np.array([0.5, 0.7])

  def lse(**kw):
    a = logw + scipy.stats.norm.logpdf(kw['x'], mu[:, 0], sd) + \
        scipy.stats.norm.logpdf(kw['y'], mu[:, 1], sd)
    return scipy.special.logsumexp(a)
  process.set_prob(lse, pscale='log')
  tg = process.lower()['target']
  assert tg['kind'] == 'gmm'
  np.testing.assert_array_equal(tg['mu'], mu)
  np.testing.assert_array_equal(tg['logw'], logw)

  def bad_sd(**kw):
    a = logw + scipy.stats.norm.logpdf(kw['x'], mu[:, 0], sd) + \
        scipy.stats.norm.logpdf(kw['y'], mu[:, 1], 2 * sd)
    m = np.max(a)
    return m + np.log(np.sum(np.exp(a - m)))

  def no_shift(**kw):
    a = logw + scipy.stats.norm.logpdf(kw['x'], mu[:, 0], sd) + \
        scipy.stats.norm.logpdf(kw['y'], mu[:, 1], sd)
    return np.log(np.sum(np.exp(a)))

  def swapped(**kw):
    a = logw + scipy.stats.norm.logpdf(kw['y'], mu[:, 1], sd) + \
        scipy.stats.norm.logpdf(kw['x'], mu[:, 0], sd)
    m = np.max(a)
    return m + np.log(np.sum(np.exp(a - m)))
  for fn in (bad_sd, no_shift, swapped):
    process.set_prob(fn, pscale='log')
    with pytest.raises(pb.NotLowerable):
      process.lower()


@pytest.mark.gpu
@pytest.mark.parametrize('name', ['mcmc_prob6', 'diag10', 'metrohast_norm1d',
                                  'mcmc_prob2'])
def test_summary_o_q_r_match_reference(name):
  """SP(samples).o / .q / .r (sp.py:160-191) against the reference's own
  summary of the same seeded chain (tools/gen_summary_golden.py): o is the
  last accepted state from step 2 on, q the transition PD over (x', x) with
  the tran's value, r (asymmetric trans) its reverse with the same value.
  The reference's o / p also carry the iid data key as a set of sizes; the
  variable keys are compared."""
  import json
  import os
  g = np.load(os.path.join(os.path.dirname(__file__), 'golden',
                           'summary_oqr.npz'))
  meta = json.loads(str(g['meta']))[name]
  builder, params, n, t, seed0 = WORKLOADS[name]
  process, init, extra, kwds, keys, _ = _build(name)
  np.random.seed(meta['seed'])
  args = (init,) if extra is None else (init, extra)
  summary = process(process.walk(process.sampler(*args, stop=meta['steps'],
                                                 **kwds)))
  for f, fkeys in meta['fields'].items():
    d = getattr(summary, f)
    if fkeys is None:
      assert d is None, f
      continue
    assert list(d.keys()) == fkeys, (f, list(d.keys()))
    for k in fkeys:
      ref = g['{}/{}/{}'.format(name, f, k)]
      assert _golden_rtol(np.ravel(d[k]), ref) <= 1e-12, (f, k)
    ref = g['{}/{}/prob'.format(name, f)]
    assert _golden_rtol(np.ravel(d.prob), ref) <= 1e-12, (f, 'prob')


@pytest.mark.gpu
@pytest.mark.parametrize('name', ['diag10', 'gibbs8', 'metrohast_norm1d'])
@pytest.mark.parametrize('stop', [None, 7])
def test_walk_hands_out_what_next_does(name, stop):
  """SP.walk's bulk hand-out (Sampler._bulk_steps) against one next() per
  step on a twin sampler: the same records, counters and last state, for a
  bounded sampler walked whole and cut at a stop, with thin > 1, and the
  sampler continuing after the walk."""
  builder, params, n, t, seed0 = WORKLOADS[name]
  process, init, extra, kwds, keys, g = _build(name)
  args = (init,) if extra is None else (init, extra)
  thin = 1 if name == 'gibbs8' else 2
  a = process.sampler(*args, stop=2 * t, chains=n, seeds=g['seeds'], thin=thin, **kwds)
  b = process.sampler(*args, stop=2 * t, chains=n, seeds=g['seeds'], thin=thin, **kwds)
  wa = list(process.walk(a, stop=stop))
  wb = []
  for s in b:
    if stop is not None and len(wb) >= stop:
      break
    wb.append(s)
  assert len(wa) == len(wb)
  assert process.get_counter(a) == process.get_counter(b)
  for sa, sb in zip(wa, wb):
    for k in keys:
      np.testing.assert_array_equal(np.asarray(sa.v[k]), np.asarray(sb.v[k]))
  la, lb = process.get_last(a), process.get_last(b)
  assert (la is None) == (lb is None)   # a walk to the end resets (sp_utils.py:14-16)
  for k in keys if la is not None else ():
    np.testing.assert_array_equal(np.asarray(la.p[k]), np.asarray(lb.p[k]))
  if stop is not None:   # both continue from the step handed out last
    na, nb = next(a), next(b)
    for k in keys:
      np.testing.assert_array_equal(np.asarray(na.v[k]), np.asarray(nb.v[k]))
  a.close()
  b.close()


@pytest.mark.gpu
def test_engines_reusing_cached_buffers_run_the_same_chains():
  """A destroyed engine's buffers and stream serve the next engine
  (pbh_cache_*): cached memory holds the old engine's data, and a run on it
  equals a run on fresh memory bit for bit."""
  from probayes_amd import Engine
  import bench
  out = []
  for rep in range(3):
    eng = Engine(bench.cfg2_spec())
    eng.init_chains(np.zeros((1000, 10)))
    eng.set_rng('philox', seed=11)
    eng.alloc_trace(40, 1)
    eng.run(40, steps_per_launch=16)
    out.append(eng.trace())
    if rep == 0:
      eng.close()
      Engine.cache_release()       # the second engine starts from fresh memory
    else:
      eng.close()                   # the third takes the second's buffers
  idle, hits, misses = Engine.cache_info()
  assert hits > 0 and idle > 0
  for k in out[0]:
    if out[0][k] is not None:
      np.testing.assert_array_equal(np.asarray(out[0][k]), np.asarray(out[1][k]))
      np.testing.assert_array_equal(np.asarray(out[0][k]), np.asarray(out[2][k]))
