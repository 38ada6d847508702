"""The SP generator API beyond walk(): SP.next / SP.reset / get_last /
get_counter / get_sampler and unbounded samplers (sampler(stop=None)),
probayes sp.py:113-128, 201-278 and sp_utils.py:8-16.

GPU tests reproduce reference chains (the golden recordings) through next()
calls and through unbounded samplers cut by walk(stop=), including where the
global NumPy legacy stream is left; interleaved draws of the caller from the
global stream are checked against the oracle fed the same interleaving.  The
production RNGs are checked for exact continuation across reset(reset_last=
False), whatever the engine computed ahead."""
import numpy as np
import pytest

import oracle
import probayes_amd as pb
from mcmc_examples import WORKLOADS, TFUN_WORKLOADS
from oracle.workloads import golden_init

ALL = dict(WORKLOADS, **TFUN_WORKLOADS)


def _build(name):
  builder, params, n, t, seed0 = ALL[name]
  g = oracle.load_golden(name)
  if params and name not in TFUN_WORKLOADS:
    params = oracle.workloads.golden_params(g)
  process, init, extra, kwds, keys = builder(pb, params)
  args = (init,) if extra is None else (init, extra)
  return process, args, kwds, keys, g, t


def _rtol(a, b):
  return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1.)))


def _stream_after(name, g, c, n_steps):
  """The value the global stream gives next after the reference drew
  n_steps steps from np.random.seed(seeds[c])."""
  if name in TFUN_WORKLOADS:   # cond_reg: gamma(31) on y_sigma steps
    rs = np.random.RandomState(int(g['seeds'][c]))
    for s in range(n_steps):
      rs.standard_gamma(31.) if s % 3 == 2 else rs.standard_normal()
    return rs.random_sample()
  states = []
  spec = oracle.golden_spec(name, g)
  oracle.legacy_streams(spec, g['seeds'][c:c + 1], n_steps, states=states)
  return states[0].random_sample()


def test_registry_without_running():
  """sampler() registers (counter 0, last None); get_sampler by index;
  reset() empties the registry -- nothing runs on the device."""
  process, args, kwds, keys, g, t = _build('metrohast_norm1d')
  s0 = process.sampler(*args, stop=5, **kwds)
  s1 = process.sampler(*args, **kwds)
  assert process.get_sampler(0) is s0 and process.get_sampler(1) is s1
  assert process.get_sampler(s1) is s1
  assert process.get_counter(s0) == 0 and process.get_last(1) is None
  assert s1.stop is None and s0.stop == 5
  process.reset()
  assert process.get_sampler() == []
  # a lone positional int is the stop (sp.py:265-267)
  s2 = process.sampler(7)
  assert s2.stop == 7 and s2.init is None


@pytest.mark.gpu
@pytest.mark.parametrize('name', ['metrohast_norm1d', 'mcmc_prob6', 'gibbs_norm2d',
                                  'gibbs_linreg'])
def test_next_calls_reproduce_the_reference_chain(name):
  """SP.next(sampler) step by step on the global stream: the reference's
  chain, the counter, get_last, and the global stream left where the
  reference leaves it."""
  process, args, kwds, keys, g, t = _build(name)
  t = min(t, 60)
  np.random.seed(int(g['seeds'][0]))
  sm = process.sampler(*args, **kwds)      # unbounded: next() drives it
  steps = [process.next(sm) for _ in range(t)]
  assert process.get_counter(sm) == t
  for i, k in enumerate(keys):
    got = np.array([s.v[k] for s in steps])
    assert _rtol(got, g['v_x'][0, :t, i]) <= 1e-12
  got = np.array([s.v.prob for s in steps])
  assert _rtol(got, g['v_p'][0, :t]) <= 1e-12
  last = process.get_last(sm)
  assert last.p[keys[0]] == steps[-1].v[keys[0]]
  assert np.random.random_sample() == _stream_after(name, g, 0, t)


@pytest.mark.gpu
@pytest.mark.parametrize('name,chunk', [('metrohast_norm1d', 7), ('diag10', 5),
                                        ('gibbs_norm2d', 3), ('gibbs_linreg', 4)])
def test_unbounded_sampler_cut_by_walk(name, chunk):
  """sampler(stop=None) in chunks, cut by walk(stop=k): the first k steps
  of the reference's chain; the walk drew k + 1 steps (it checks after each
  sample), and so did the global stream."""
  process, args, kwds, keys, g, t = _build(name)
  k = min(t, 40) - 1
  np.random.seed(int(g['seeds'][1]))
  sm = process.sampler(*args, chunk=chunk, **kwds)
  samples = process.walk(sm, stop=k)
  assert len(samples) == k
  summary = process(samples)
  for i, key in enumerate(keys):
    assert _rtol(np.asarray(summary.v[key]), g['v_x'][1, :k, i]) <= 1e-12
  assert process.get_counter(sm) == k + 1
  assert np.random.random_sample() == _stream_after(name, g, 1, k + 1)


@pytest.mark.gpu
def test_caller_draws_between_steps_are_seen_as_the_reference_sees_them():
  """The sampler draws the global stream ahead; a caller drawing from it
  between two next() calls takes numbers the reference would have given to
  the caller, so the steps drawn ahead are discarded and redrawn: the chain
  equals the oracle fed that interleaving."""
  name = 'metrohast_norm1d'
  process, args, kwds, keys, g, t = _build(name)
  spec = oracle.golden_spec(name, g)
  seed, T = int(g['seeds'][0]), 24
  # the reference's interleaving, on the host
  rs = np.random.RandomState(seed)
  streams = np.empty((T, oracle.stream_width(spec), 1))
  user = []
  kind = spec['proposal']['kind']
  assert kind in ('gauss', 'sphere')   # metrohast_norm1d: the tuple delta
  for s in range(T):
    # oracle/streams.py's per-step order: the proposal's draws, then t
    streams[s, :-1, 0] = (rs.standard_normal(spec['dim']) if kind == 'gauss'
                          else rs.random_sample(spec['dim']))
    streams[s, -1, 0] = rs.random_sample()
    if s % 5 == 2:
      user.append(rs.random_sample())
  ref = oracle.run_mh(spec, golden_init(name, 1), streams)
  np.random.seed(seed)
  sm = process.sampler(*args, chunk=64, **kwds)
  got, mine = [], []
  for s in range(T):
    got.append(process.next(sm).v[keys[0]])
    if s % 5 == 2:
      mine.append(np.random.random_sample())
  assert mine == user
  assert _rtol(np.array(got), ref['v_x'][0, :, 0]) <= 1e-12
  assert np.random.random_sample() == rs.random_sample()


@pytest.mark.gpu
def test_bounded_generator_resets_at_its_stop():
  """sp_utils.py:13-16: when the counter reaches stop the generator ends
  and resets the sampler (counter 0, last None); the next SP.next restarts
  the chains at init (step 1 again: o is None, every chain accepts)."""
  process, args, kwds, keys, g, t = _build('diag10')
  sm = process.sampler(*args, stop=12, chains=64, rng='philox', seed=3, **kwds)
  steps = list(sm)
  assert len(steps) == 12
  assert process.get_counter(sm) == 0 and process.get_last(sm) is None
  assert list(sm) == []                       # an exhausted generator
  s1 = process.next(sm)
  assert s1.o is None and np.all(s1.u)
  assert process.get_counter(sm) == 1


@pytest.mark.gpu
@pytest.mark.parametrize('rng,seeds', [('philox', None), ('xoshiro', None),
                                       ('legacy', True)])
def test_reset_keeps_or_restarts_the_chains(rng, seeds):
  """reset(reset_last=False) continues the chains from the last step handed
  out -- exactly the uninterrupted run, although the engine computed ahead
  (counter-based Philox; the xoshiro and device legacy streams are rewound);
  reset(reset_last=True) restarts them at init with step 1's auto-accept."""
  name = 'diag10'
  process, args, kwds, keys, g, t = _build(name)
  n = 48
  opts = dict(chains=n, rng=rng, seed=11, chunk=16, **kwds)
  if seeds:
    opts['seeds'] = g['seeds'][:1].repeat(n) + np.arange(n)
  ref = process.sampler(*args, **opts)
  want = [process.next(ref).v[keys[0]] for _ in range(30)]
  sm = process.sampler(*args, **opts)
  got = [process.next(sm).v[keys[0]] for _ in range(9)]
  process.reset(sm, reset_last=False)
  assert process.get_counter(sm) == 0
  got += [process.next(sm).v[keys[0]] for _ in range(21)]
  np.testing.assert_array_equal(np.array(got), np.array(want))
  process.reset(sm)                               # reset_last=True
  s1 = process.next(sm)
  assert s1.o is None and np.all(s1.u)
  assert process.get_counter(sm) == 1


@pytest.mark.gpu
def test_summary_spans_blocks():
  """SP(samples) over steps from several engine blocks equals the summary
  of the same steps computed in one block (o, p, v, u)."""
  process, args, kwds, keys, g, t = _build('metrohast_norm1d')
  np.random.seed(int(g['seeds'][0]))
  a = process(process.walk(process.sampler(*args, stop=30, **kwds)))
  np.random.seed(int(g['seeds'][0]))
  b = process(process.walk(process.sampler(*args, chunk=4, **kwds), stop=30))
  for key in keys:
    np.testing.assert_array_equal(np.asarray(a.v[key]), np.asarray(b.v[key]))
    np.testing.assert_array_equal(np.asarray(a.o[key]), np.asarray(b.o[key]))
    np.testing.assert_array_equal(np.asarray(a.p[key]), np.asarray(b.p[key]))
  assert a.u == b.u


@pytest.mark.gpu
def test_interleaved_bounded_samplers_cost_linear_draw_ahead():
  """two bounded samplers on the global stream, stepped in
  turn.  Each one's draws interleave with the other's in NumPy's global
  state, so every step of one invalidates what the other drew ahead; the
  draw-ahead falls back to one step after such a rewind (then doubles), so
  the steps computed stay O(stop) per sampler, and both chains equal the
  oracle fed the same interleaved stream."""
  name = 'metrohast_norm1d'
  process, args, kwds, keys, g, t = _build(name)
  spec = oracle.golden_spec(name, g)
  seed, T = int(g['seeds'][0]), 150
  rs = np.random.RandomState(seed)
  w = oracle.stream_width(spec)
  streams = np.empty((2, T, w, 1))
  for s in range(T):
    for c in range(2):   # A's step s, then B's step s
      streams[c, s, :-1, 0] = rs.random_sample(spec['dim'])
      streams[c, s, -1, 0] = rs.random_sample()
  refs = [oracle.run_mh(spec, golden_init(name, 1), streams[c]) for c in range(2)]
  np.random.seed(seed)
  a = process.sampler(*args, stop=T, **kwds)
  b = process.sampler(*args, stop=T, **kwds)
  got = [[], []]
  for s in range(T):
    got[0].append(process.next(a).v[keys[0]])
    got[1].append(process.next(b).v[keys[0]])
  for c in range(2):
    assert _rtol(np.array(got[c]), refs[c]['v_x'][0, :, 0]) <= 1e-12
  assert a.n_computed <= 3 * T and b.n_computed <= 3 * T, (a.n_computed, b.n_computed)
  assert np.random.random_sample() == rs.random_sample()


def test_samplers_are_not_kept_alive_by_the_registry():
  """SP's counters and last states hold their samplers weakly;
  after SP.reset() empties the registry, a sampler the caller dropped is
  collected (and with it its engine's device buffers)."""
  import gc
  import weakref
  process, args, kwds, keys, g, t = _build('metrohast_norm1d')
  sm = process.sampler(*args, stop=5, **kwds)
  process._counter[sm] += 3
  assert process.get_counter(sm) == 3
  ref = weakref.ref(sm)
  process.reset()
  del sm
  gc.collect()
  assert ref() is None
  assert len(process.get_counter()) == 0 and len(process.get_last()) == 0


def _registry_fn(name):
  """A stand-in with the identity of the reference registry's function
  (probayes/sp_utils.py:19-85): the façade recognises it by module and name."""
  def f(*args, **kwds):
    raise AssertionError('never called: the kernel runs the sampler')
  f.__name__ = name
  f.__module__ = 'probayes.sp_utils'
  return f


def _same_spec(a, b):
  if isinstance(a, dict):
    return isinstance(b, dict) and a.keys() == b.keys() and \
        all(_same_spec(a[k], b[k]) for k in a)
  if isinstance(a, (list, tuple)):
    return len(a) == len(b) and all(_same_spec(x, y) for x, y in zip(a, b))
  if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
    return np.array_equal(np.asarray(a), np.asarray(b), equal_nan=True)
  return a == b or (a != a and b != b)


def test_registry_functions_as_objects():
  """set_scores / set_thresh / set_update with the registry's own functions
  passed as objects (sp.py:57-100 wraps them as Expressions): they lower as
  their names when the scores' pscale keyword matches the model's; with
  pscale=None the reference divides the log-probabilities as linear ones
  (pscales.py:27-28, 219-236), which has no kernel form; the function object
  does not set thresh and update, so they must be given; any other callable
  still has no kernel."""
  process, args, kwds, keys, g, t = _build('metrohast_norm1d')
  extra = args[1] if len(args) > 1 else None
  ref = process.lower(extra, kwds.get('iid', False), kwds.get('joint', False))
  process.set_scores(_registry_fn('hastings_scores'), pscale='log')
  process.set_thresh(_registry_fn('hastings_thresh'))
  process.set_update(_registry_fn('metropolis_update'))
  spec = process.lower(extra, kwds.get('iid', False), kwds.get('joint', False))
  assert _same_spec(spec, ref)
  process.set_scores(_registry_fn('hastings_scores'))      # pscale=None
  with pytest.raises(pb.NotLowerable):
    process.lower(extra, kwds.get('iid', False), kwds.get('joint', False))
  fresh, *_ = _build('metrohast_norm1d')
  fresh.set_thresh(None)
  fresh.set_update(None)
  fresh.set_scores(_registry_fn('hastings_scores'), pscale='log')
  with pytest.raises(pb.NotLowerable):                     # no thresh / update
    fresh.lower(extra, kwds.get('iid', False), kwds.get('joint', False))
  with pytest.raises(pb.NotLowerable):
    process.set_scores(lambda opqr: 1.)
  with pytest.raises(pb.NotLowerable):
    process.set_thresh(_registry_fn('hastings_scores'))    # the wrong slot


def test_registry_name_cascade_overwrites():
  """sp.py:57-66, 74-83: set_scores(name) overwrites thresh and update
  (through set_thresh), set_thresh(name) overwrites update; a registry name
  with arguments is an AssertionError; set_scores(None) clears the scores
  only."""
  process, args, kwds, keys, g, t = _build('metrohast_norm1d')
  extra = args[1] if len(args) > 1 else None
  lw = lambda p: p.lower(extra, kwds.get('iid', False), kwds.get('joint', False))
  ref = lw(process)
  process.set_update('gibbs')
  process.set_thresh('gibbs')
  process.set_scores('hastings')          # the reference runs Hastings
  assert process._thresh == 'hastings' and process._update == 'hastings'
  assert _same_spec(lw(process), ref)
  process.set_update('gibbs')
  process.set_thresh('hastings')          # overwrites the update again
  assert process._update == 'hastings'
  assert _same_spec(lw(process), ref)
  process.set_scores(None)
  assert process._thresh == 'hastings' and process._update == 'hastings'
  for setter in (process.set_scores, process.set_thresh, process.set_update):
    with pytest.raises(AssertionError):
      setter('hastings', 1.)
    with pytest.raises(AssertionError):
      setter('metropolis', pscale='log')


def test_registry_functions_with_arguments_refused():
  """A registry function object wrapped with arguments computes something
  else in the reference (Expression(fn, *args, **kwds), sp.py:67, 84, 100):
  thresh with limits draws np.random.uniform(lo, hi); scores with a
  positional pscale; these raise NotLowerable instead of lowering silently.
  A function from another module named sp_utils is a custom callable."""
  process, *_ = _build('metrohast_norm1d')
  with pytest.raises(pb.NotLowerable):
    process.set_thresh(_registry_fn('metropolis_thresh'), 0.2, 0.9)
  with pytest.raises(pb.NotLowerable):
    process.set_thresh(_registry_fn('hastings_thresh'), low=0.2)
  with pytest.raises(pb.NotLowerable):
    process.set_scores(_registry_fn('metropolis_scores'), 'log')
  with pytest.raises(pb.NotLowerable):
    process.set_update(_registry_fn('hastings_update'), 1)
  process.set_scores(_registry_fn('metropolis_scores'), pscale='log')
  assert process._scores == 'metropolis' and process._scores_pscale == 'log'
  imposter = _registry_fn('metropolis_scores')
  imposter.__module__ = 'myproj.sp_utils'
  with pytest.raises(pb.NotLowerable):
    process.set_scores(imposter, pscale='log')
