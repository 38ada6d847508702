"""SP: the stochastic-process facade (mirrors probayes sp.py / sd.py).

The calls examples/mcmc makes -- SP(...), set_prob, set_tran, set_delta,
set_scores, set_thresh, set_update, Delta, sampler, walk, SP(samples) and the
summary fields v[key], v.prob, v.rescaled(), u.count(True) -- keep their
reference meaning.  Underneath, a sampler lowers the model to a kernel spec
(probayes_amd.lower) and runs every step of every chain in the HIP engine;
the reference's per-step Python call stack never runs.

Extensions over the reference (keyword-only, defaults keep its behaviour):
  chains=N   run N independent chains in one batch (values become [T, N]);
  rng=       'legacy' (default for one chain: NumPy's GLOBAL legacy stream,
             exactly as the reference draws it, so seeded scripts reproduce
             the reference's chains), 'legacy' with seeds=[...] (chain c uses
             RandomState(seeds[c])), 'philox' (production, seed=) or
             'philox_f64';
  device=, thin=, steps_per_launch=.
"""
import collections

import numpy as np
import scipy.stats

from probayes_amd import lower as L
from probayes_amd import replay
from probayes_amd.engine import Engine
from probayes_amd.pd import PD
from probayes_amd.pscales import is_log
from probayes_amd.rv import RF, RV

MCMC_SAMPLERS = ('metropolis', 'hastings', 'gibbs')   # sp_utils.py:87-91


class FlagArray(np.ndarray):
  """Update flags u with the list API the examples use (u.count(True))."""

  def count(self, value=True):
    return int(np.sum(self == bool(value)))


def _as_rf(a):
  if isinstance(a, RF):
    return a
  if isinstance(a, RV):
    return RF(a)
  raise TypeError('SP takes RVs or RFs, not {}'.format(type(a)))


def _key(k):
  return k.name if isinstance(k, RV) else str(k)


class SP:
  """A stochastic process over the roots' variables (sp.py:14)."""

  def __init__(self, *args):
    rfs = [_as_rf(a) for a in args]
    if len(rfs) == 1:
      self.leafs, self.roots = None, rfs[0]
    elif len(rfs) == 2:
      self.leafs, self.roots = rfs
    else:
      raise NotImplementedError('SP takes one RF or (stats, paras)')
    self.Delta = self.roots.Delta
    self._prob = None
    self._tran = None      # (tran, args, kwds) or an RF to delegate to
    self._delta = None     # (delta, args, kwds) or an RF
    self._tfun = None
    self._scores = self._thresh = self._update = None

  # ---- specification (sp.py:57-100, rf.py:91-304, field.py:220-317) -----
  @property
  def keylist(self):
    return self.roots.keylist

  def set_prob(self, prob=None, *args, **kwds):
    self._prob = (prob, args, dict(kwds))

  def _subfield(self, spec):
    """dependence.py:316-326: an RF of this process or its subfield name
    ('leafs' for a one-field SP; 'leafs' / 'roots' for SP(leafs, roots))."""
    if isinstance(spec, RF):
      return spec
    if isinstance(spec, str):
      fields = {'leafs': self.roots} if self.leafs is None else \
          {'leafs': self.leafs, 'roots': self.roots}
      if spec not in fields:
        raise AssertionError('{} absent from {}'.format(spec, self.roots))
      return fields[spec]
    return None

  def set_tran(self, tran=None, *args, **kwds):
    """sd.py:97-105.  An RF (or its subfield name) lends its tran and tfun;
    the process's own _sym_tran is then left unset, so hastings takes the
    reverse branch with r = q (sd.py:276-277, rf.py:536)."""
    if isinstance(tran, np.ndarray):
      # dependence.py:320 compares the array with the subfields and raises
      raise ValueError('The truth value of an array with more than one '
                       'element is ambiguous. Use a.any() or a.all()')
    sub = self._subfield(tran)
    self._tran = sub if sub is not None else (tran, args, dict(kwds))

  def set_delta(self, delta=None, *args, **kwds):
    """dependence.py:329-339: an RF (or its subfield name) lends its delta."""
    sub = self._subfield(delta)
    self._delta = sub if sub is not None else (delta, args, dict(kwds))

  def set_tfun(self, tfun=None, *args, **kwds):
    self._tfun = tfun

  def set_scores(self, scores=None, *args, **kwds):
    self._scores = scores
    if scores in MCMC_SAMPLERS:
      self._thresh = self._thresh or scores
      self._update = self._update or scores
    elif scores is not None:
      raise L.NotLowerable('custom scores callables have no kernel')

  def set_thresh(self, thresh=None, *args, **kwds):
    if thresh is not None and thresh not in MCMC_SAMPLERS:
      raise L.NotLowerable('custom thresh callables have no kernel')
    self._thresh = thresh

  def set_update(self, update=None, *args, **kwds):
    if update is not None and update not in MCMC_SAMPLERS:
      raise L.NotLowerable('custom update callables have no kernel')
    self._update = update

  # ---- lowering -----------------------------------------------------------
  def _pscale(self, kw_pscale):
    if kw_pscale is not None:
      return 'log' if is_log(kw_pscale) else 'lin'
    rvs = list(self.roots.rvs) + (list(self.leafs.rvs) if self.leafs else [])
    return 'log' if any(is_log(v.pscale) for v in rvs) else 'lin'

  def _lower_target(self, extra, iid):
    if self._prob is None:
      raise L.NotLowerable('set_prob() first')
    prob, args, kwds = self._prob
    kwds = dict(kwds)
    pscale_kw = kwds.pop('pscale', None)
    order = kwds.pop('order', None)
    names = self.keylist
    if hasattr(prob, 'pbh_target'):
      return dict(prob.pbh_target), pscale_kw or prob.pbh_pscale
    if prob is scipy.stats.multivariate_normal:
      if len(args) < 2:
        raise L.NotLowerable('multivariate_normal needs (mean, cov)')
      return {'kind': 'mvn', 'mean': np.asarray(args[0], np.float64),
              'cov': np.asarray(args[1], np.float64)}, self._pscale(pscale_kw)
    is_logpdf = L.is_same_callable(prob, scipy.stats.norm.logpdf)
    is_pdf = L.is_same_callable(prob, scipy.stats.norm.pdf)
    is_updf = L.is_same_callable(prob, scipy.stats.uniform.pdf)
    if is_logpdf or is_pdf or is_updf:
      order = order or {names[0]: 0}
      slot = {}
      for k, v in order.items():
        slot[v] = _key(k)
      loc = kwds.get('loc', args[0] if len(args) > 0 else 0.)
      scale = kwds.get('scale', args[1] if len(args) > 1 else 1.)
      xname = slot.get(0)
      if 'loc' in slot or 'scale' in slot:
        # data variable at position 0, roots as loc / scale (iid product)
        if not (is_logpdf and iid and extra and xname in extra):
          raise L.NotLowerable('norm density over data needs logpdf, iid=True '
                               'and the data in extra')
        return {'kind': 'norm_iid',
                'obs': np.asarray(extra[xname], np.float64).reshape(-1),
                'loc': names.index(slot['loc']),
                'scale': names.index(slot['scale'])}, self._pscale(pscale_kw)
      if len(names) != 1 or xname != names[0]:
        raise L.NotLowerable('scipy density form needs a single variable')
      loc, scale = np.array([float(loc)]), np.array([float(scale)])
      if is_logpdf:
        return {'kind': 'diag_gauss', 'mu': loc, 'sigma': scale}, \
            self._pscale(pscale_kw)
      if is_pdf:
        return {'kind': 'norm_pdf', 'loc': loc, 'scale': scale}, \
            self._pscale(pscale_kw)
      return {'kind': 'uniform_pdf', 'lo': loc, 'scale': scale}, \
          self._pscale(pscale_kw)
    if callable(prob):
      try:
        target, ps = L.trace_prob(prob, names)
      except L.NotLowerable as e:
        try:
          target, ps = L.trace_logsumexp(prob, names)
        except L.NotLowerable:
          raise e
      return target, (self._pscale(pscale_kw) if pscale_kw else ps)
    raise L.NotLowerable('density {} is not a recognised form'.format(prob))

  def _tran_spec(self):
    src = self._tran
    if isinstance(src, RF):
      src = src.tran
    return src

  def _delta_spec(self):
    src = self._delta
    if isinstance(src, RF):
      return src.delta, src.delta_args, src.delta_kwds
    return src if src is not None else (None, (), {})

  def lower(self, extra=None, iid=False, joint=False):
    """The kernel spec of this process (probayes_amd/spec.py)."""
    from probayes_amd.spec import make_spec
    if self._tfun is not None:
      return self._lower_linreg(extra, iid, joint)
    names, rvs = self.keylist, self.roots.rvs
    d = len(names)
    extra = {_key(k): v for k, v in (extra or {}).items()}
    target, pscale = self._lower_target(extra, iid)
    scores = self._scores
    if scores not in MCMC_SAMPLERS:
      raise L.NotLowerable('set_scores() to one of {}'.format(MCMC_SAMPLERS))
    # metropolis_/hastings_ thresh and update are the same functions
    # (sp_utils.py:30-37,67-72); gibbs pairs only with gibbs.
    ok = ('gibbs',) if scores == 'gibbs' else ('metropolis', 'hastings')
    if self._update not in (None,) + ok or self._thresh not in (None,) + ok:
      raise L.NotLowerable('mixed scores/thresh/update samplers')
    prior = None
    if joint and any(rv.vtype is int for rv in rvs):
      raise L.NotLowerable('joint=True priors of int variables (a uniform '
                           'over the value set) have no kernel')
    if joint:
      lens = [rv.length for rv in rvs]
      nl = [-np.log(L_) if np.isfinite(L_) else -np.inf for L_ in lens]
      logp = nl[0]
      for v in nl[1:]:
        logp = logp + v                               # prod_rule order
      prior = {'lo': [rv.vlims[0] for rv in rvs],
               'hi': [rv.vlims[1] for rv in rvs],
               'lo_incl': [int(rv.lo_incl) for rv in rvs],
               'hi_incl': [int(rv.hi_incl) for rv in rvs],
               'logp': float(logp)}
    ufun = [int(rv.log_ufun) for rv in rvs]
    tran = self._tran_spec()
    if scores == 'gibbs':
      t, targs, tkw = tran if tran else (None, (), {})
      if t is not scipy.stats.multivariate_normal or len(targs) < 2:
        raise L.NotLowerable('gibbs needs set_tran(multivariate_normal, mean, '
                             'cov, tsteps=...)')
      proposal = {'kind': 'gibbs', 'mean': targs[0], 'cov': targs[1],
                  'lo': [rv.vlims[0] for rv in rvs],
                  'hi': [rv.vlims[1] for rv in rvs],
                  # rf.py:446-452: tsteps None/0 updates every coordinate
                  'tsteps': int(tkw.get('tsteps') or d)}
      return make_spec(d, target, proposal, scores='gibbs', pscale=pscale,
                       prior=prior, ufun=ufun, names=names)
    proposal = self._lower_delta(rvs, names)
    lud = self._tran.lud if isinstance(self._tran, RF) else None
    if lud is not None:
      proposal['tfun'] = lud
    tran_spec = self._lower_tran(tran, names, scores,
                                 via_rf=isinstance(self._tran, RF))
    return make_spec(d, target, proposal, scores=scores, pscale=pscale,
                     tran=tran_spec, prior=prior, ufun=ufun, names=names)

  def _lower_linreg(self, extra, iid, joint):
    """User-tfun Gibbs (rf.py:413-462): lowered when the paras RF's tfun is
    a linreg.LinRegConditional over beta_0 & beta_1 & y_sigma with tsteps=1,
    gibbs scores, and a density equal to norm.logpdf(y, b0 + b1 x, y_sigma)
    over the iid data in `extra` (examples/mcmc/gibbs_linreg.py)."""
    from probayes_amd import linreg
    rf = self._subfield(self._tfun) or self._tfun
    tf = getattr(rf, 'tfun', None)
    if tf is None or not callable(tf[0]):
      raise L.NotLowerable('user tfun Gibbs needs a callable conditional')
    cond, _, tkw = tf
    if tuple(rf.keylist) != linreg.KEYS or tuple(self.keylist) != linreg.KEYS:
      raise L.NotLowerable('linreg Gibbs needs paras beta_0 & beta_1 & y_sigma')
    if int(tkw.get('tsteps') or 0) != 1:
      raise L.NotLowerable('linreg Gibbs needs tsteps=1')
    if self._scores != 'gibbs' or not iid:
      raise L.NotLowerable("linreg Gibbs needs set_scores('gibbs') and iid=True")
    if self.leafs is None or tuple(self.leafs.keylist) != ('x', 'y'):
      raise L.NotLowerable('linreg Gibbs needs SP(x & y, paras)')
    ex = {_key(k): v for k, v in (extra or {}).items()}
    if 'x,y' in ex:
      x_obs, y_obs = (np.asarray(v, np.float64) for v in ex['x,y'])
    elif 'x' in ex and 'y' in ex:
      x_obs, y_obs = np.asarray(ex['x'], np.float64), np.asarray(ex['y'], np.float64)
    else:
      raise L.NotLowerable("linreg Gibbs needs the data as extra {'x,y': ...}")
    for k, v in (('x', x_obs), ('y', y_obs)):
      if k not in tkw or not np.array_equal(np.asarray(tkw[k], np.float64), v):
        raise L.NotLowerable('the tfun data must be the sampler data')
    if isinstance(cond, linreg.LinRegConditional):
      if cond.n_obs != len(x_obs):
        raise L.NotLowerable('LinRegConditional n_obs != the data size')
      hyper = cond.hyper
    else:   # the user's own cond_reg, identified by probing
      hyper = linreg.identify_conditional(cond, x_obs, y_obs)
    if self._prob is None:
      raise L.NotLowerable('set_prob() first')
    prob, pargs, pkw = self._prob
    pkw = dict(pkw)
    pscale = pkw.pop('pscale', None)
    if pargs or pkw or not is_log(pscale) or \
        not linreg.identify_loglik(prob, x_obs, y_obs):
      raise L.NotLowerable('linreg Gibbs needs the log density '
                           'norm.logpdf(y, beta_0 + beta_1*x, y_sigma)')
    rvs = self.roots.rvs
    if joint and not all(rv.lo_incl and rv.hi_incl for rv in rvs):
      raise L.NotLowerable('linreg Gibbs priors need closed (list) vsets')
    vsets = [tuple(rv.vlims) for rv in rvs] if joint else None
    return {'kind': 'linreg', 'names': list(linreg.KEYS), 'pscale': 'log',
            'x_obs': x_obs, 'y_obs': y_obs, 'hyper': hyper,
            'vsets': vsets}

  def _lower_delta(self, rvs, names):
    """Field.set_delta / eval_delta / apply_delta (field.py:220-317,
    469-552; variable.py:600-739) lowered to a proposal spec."""
    delta, dargs, dkw = self._delta_spec()
    if delta is None:
      raise L.NotLowerable('set_delta() first')
    if callable(delta) and not isinstance(delta, tuple):
      if dkw:   # the reference hands these keywords to the callable itself
        raise L.NotLowerable('keywords of a callable delta ({}) are the '
                             "callable's own".format(sorted(dkw)))
      return L.trace_delta(delta, names)
    scale = bool(dkw.get('scale', False))
    bound = bool(dkw.get('bound', False))
    lengths = np.array([rv.length for rv in rvs], np.float64)
    is_int = np.array([rv.vtype is int for rv in rvs])
    d = len(rvs)
    on = np.ones(d, np.int32)
    if isinstance(delta, dict):
      # field.py:261-263 converts the dict to a Delta but tests the ORIGINAL
      # argument against the Delta type, so a dict takes the tuple branch
      # (:308-316): no variable delta is set, eval_delta yields Delta(None,
      # ...) and apply_delta returns the values unchanged, unbounded
      unknown = set(delta) - set(names)
      if unknown or len(delta) != d:
        raise TypeError('Delta() fields {} do not match {}'.format(
            sorted(delta), names))
      unscale = dargs[0] if dargs else {}
      for rv, L_ in zip(rvs, lengths):
        if rv.name not in unscale and not np.isfinite(L_):
          raise AssertionError('Cannot spherise Variable {} with infinite '
                               'length'.format(rv.name))
      return {'kind': 'vardelta', 'mode': np.zeros(d, np.int32),
              'delta': np.zeros(d)}
    if isinstance(delta, tuple) and hasattr(delta, '_fields'):
      # a Delta instance: each variable's own delta (field.py:264-274)
      if list(delta._fields) != list(names):
        raise L.NotLowerable('Delta fields {} are not the process variables '
                             '{}'.format(list(delta._fields), names))
      if dargs:
        raise AssertionError('Optional args prohibited for dict/delta '
                             'instance inputs')
      mode, steps = np.zeros(d, np.int32), np.zeros(d)
      for i, el in enumerate(delta):
        m, v = self._var_delta(el, rvs[i])
        if m is None:          # delta None: apply_delta returns the value
          on[i] = 0
          continue
        if m == 0 and scale:   # variable.py:637-639: only a bare scalar
          if not np.isfinite(lengths[i]):
            raise AssertionError('Cannot scale by infinite length')
          v = v * lengths[i]
        mode[i], steps[i] = m, v
      prop = {'kind': 'vardelta', 'mode': mode, 'delta': steps}
    elif isinstance(delta, tuple):
      # spherical (field.py:308-316, 502-531)
      unscale = dargs[0] if dargs else {}
      if unscale:
        # eval_delta then builds a Delta without the unscaled keys (or from
        # the args tuple itself) and fails
        raise TypeError('a spherical delta with unscaled variables {} is '
                        'not constructible'.format(sorted(unscale)))
      if len(delta) != 1:
        raise AssertionError('Tuple delta must contain one element')
      if not np.all(np.isfinite(lengths)):
        bad = [rv.name for rv, L_ in zip(rvs, lengths) if not np.isfinite(L_)]
        raise AssertionError('Cannot spherise Variable {} with infinite '
                             'length'.format(bad[0]))
      d0 = float(delta[0])
      if scale:
        d0 = d0 * np.sqrt(np.sum(lengths ** 2))        # field.py:513-515
        mult = lengths
      else:
        mult = np.ones(d)
      prop = {'kind': 'sphere', 'delta': d0, 'lengths': mult}
    else:
      # a bare scalar or a one-element list, per-variable overrides in
      # args[0] exempt from scaling (field.py:276-306)
      urand = isinstance(delta, list)
      if urand:
        if len(delta) != 1:
          raise AssertionError('List delta requires a single element')
        delta = delta[0]
      if len(dargs) > 1 or (dargs and not isinstance(dargs[0], dict)):
        raise AssertionError('Optional positional arguments must comprises a '
                             'single dict')
      unscale = dargs[0] if dargs else {}
      extra_keys = set(unscale) - set(names)
      if extra_keys:
        raise TypeError('unexpected Delta fields {}'.format(sorted(extra_keys)))
      mode, steps = np.zeros(d, np.int32), np.zeros(d)
      for i, rv in enumerate(rvs):
        val = unscale.get(rv.name, delta)
        if scale and rv.name not in unscale:
          if not np.isfinite(lengths[i]):
            raise AssertionError('Cannot scale by infinite length for '
                                 'Variable {}'.format(rv.name))
          val = val * lengths[i]
        m, v = self._var_delta([val] if urand else val, rvs[i])
        if m is None:
          on[i] = 0
          continue
        mode[i], steps[i] = m, v
      if urand and not is_int.any() and np.all(mode == 2):
        prop = {'kind': 'uniform', 'delta': steps}
      else:
        prop = {'kind': 'vardelta', 'mode': mode, 'delta': steps}
    if is_int.any():
      prop['vint'] = is_int.astype(np.int32)
    if bound:
      # variable.py:707-713: int limits always clamp; float tuple limits
      # are exclusive
      prop['bound'] = {
          'on': on, 'lo': np.array([rv.vlims[0] for rv in rvs], np.float64),
          'hi': np.array([rv.vlims[1] for rv in rvs], np.float64),
          'xlo': np.array([0 if rv.vtype is int else int(not rv.lo_incl)
                           for rv in rvs], np.int32),
          'xhi': np.array([0 if rv.vtype is int else int(not rv.hi_incl)
                           for rv in rvs], np.int32)}
    return prop

  @staticmethod
  def _var_delta(el, rv):
    """One variable's delta (variable.py:613-640) -> (mode, step): tuple ->
    polarity, list -> uniform (randint for an int variable), bare scalar ->
    fixed; None -> (None, 0)."""
    if el is None:
      return None, 0.
    if callable(el):
      raise L.NotLowerable('callable per-variable deltas have no kernel')
    if isinstance(el, (tuple, list)):
      if len(el) != 1:
        raise AssertionError('{} delta must contain one element'.format(
            'Tuple' if isinstance(el, tuple) else 'List'))
      v = el[0]
      if not np.isscalar(v):
        raise AssertionError('Unrecognised delta type: {}'.format(v))
      if isinstance(el, tuple):
        return 1, float(v)
      if rv.vtype is int:
        if not int(v) >= 1:    # randint(-v, v) needs trunc(v) >= 1
          raise ValueError('randint(-{0}, {0}): low >= high'.format(v))
        return 3, float(v)
      return 2, float(v)
    if not np.isscalar(el):
      raise AssertionError('Unrecognised delta type: {}'.format(el))
    return 0, float(el)

  def _lower_tran(self, tran, names, scores, via_rf=False):
    if scores == 'metropolis':
      return None
    if not tran or tran[0] is None:
      raise L.NotLowerable('hastings scores need set_tran()')
    t = tran[0]
    if isinstance(t, np.ndarray):
      # a covariance tran is not callable: eval_tran returns the default
      # conditional of the RF's pscale (rf.py:20, 510-511)
      rf = self._tran
      return {'kind': 'const', 'sym': not via_rf,
              'value': 0. if any(is_log(v.pscale) for v in rf.rvs) else 1.}
    if via_rf:
      form = L.trace_tran(t[0] if isinstance(t, tuple) else t, names)
      form['sym'] = False
      return form
    if isinstance(t, tuple):
      form = L.trace_tran(t[0], names)
      form['sym'] = False
    else:
      form = L.trace_tran(t, names)
      form['sym'] = True
    return form

  # ---- sampling (sp.py:261-295) ---------------------------------------------
  def sampler(self, *args, stop=None, iid=False, joint=False, chains=None,
              seeds=None, rng=None, seed=0, device=0, thin=1,
              steps_per_launch=0, debug=None):
    init = args[0] if args else None
    extra = args[1] if len(args) > 1 else None
    if stop is None:
      raise NotImplementedError('the GPU sampler needs stop=n_steps')
    return Sampler(self, init, extra, int(stop), iid, joint, chains, seeds,
                   rng, seed, device, thin, steps_per_launch, debug)

  def walk(self, sampler, stop=None):
    """sp.py:281-295."""
    steps = collections.deque()
    for sample in sampler:
      if stop is not None and len(steps) >= stop:
        break
      steps.append(sample)
    return steps

  def __call__(self, samples, **kwds):
    """Summary of a walk (sp.py:131-198) as trace-backed PDs.  With
    ``conditionalise=True`` the o, p and v summaries are conditionalised on
    the leaf keys (sp.py:196-197), which the reference cannot do for a
    summary (see PD.conditionalise)."""
    conditionalise = kwds.pop('conditionalise', None)
    samples = list(samples)
    if not samples or not isinstance(samples[0], Step):
      raise TypeError('SP() summarises samples from SP.sampler()')
    sm = samples[0].sampler
    idx = np.array([s.i for s in samples])
    summary = sm.summary(idx)
    if conditionalise:
      for key in ('o', 'p', 'v'):
        pd = getattr(summary, key)
        if pd is not None:
          summary = summary._replace(**{key: pd.conditionalise(list(pd.keys()))})
    return summary


OPQRSTUV = collections.namedtuple('opqrstuv', ['o', 'p', 'q', 'r', 's', 't',
                                                'u', 'v'])


class Step:
  """One recorded step of a Sampler; fields as the reference's opqrstuv
  (sp.py:257-258), built lazily from the trace arrays."""

  __slots__ = ('sampler', 'i')

  def __init__(self, sampler, i):
    self.sampler, self.i = sampler, i

  def _pd(self, xs, ps, t):
    sm = self.sampler
    vals = {k: xs[..., t, i] if sm.batched else float(xs[0, t, i])
            for i, k in enumerate(sm.names)}
    prob = ps[..., t] if sm.batched else float(ps[0, t])
    return PD('p', vals, prob=prob, pscale=sm.pscale)

  @property
  def v(self):
    return self._pd(self.sampler.tr['v_x'], self.sampler.tr['v_p'], self.i)

  @property
  def p(self):
    tr = self.sampler.tr
    if 'p_x' not in tr:
      return None
    return self._pd(tr['p_x'], tr['p_p'], self.i)

  @property
  def o(self):
    if self.i == 0:
      return None
    return self._pd(self.sampler.tr['v_x'], self.sampler.tr['v_p'], self.i - 1)

  @property
  def u(self):
    u = self.sampler.tr['u'][:, self.i].astype(bool)
    if self.sampler.batched:
      return u
    return True if u[0] else None

  @property
  def s(self):
    tr = self.sampler.tr
    if 's' not in tr:
      return None
    v = tr['s'][:, self.i]
    if self.sampler.batched:
      return v
    return None if np.isnan(v[0]) else float(v[0])

  @property
  def t(self):
    th = self.sampler.thresholds
    if th is None:
      return None
    return th[:, self.i] if self.sampler.batched else float(th[0, self.i])

  def astuple(self):
    return OPQRSTUV(self.o, self.p, None, None, self.s, self.t, self.u, self.v)

  def __getitem__(self, i):
    return self.astuple()[i]


class Sampler:
  """A lowered, batched MH/Gibbs run of `stop` steps (sp.py:261-278)."""

  def __init__(self, sp, init, extra, stop, iid, joint, chains, seeds, rng,
               seed, device, thin, steps_per_launch, debug):
    self.sp, self.init, self.extra = sp, init, extra
    self.stop, self.iid, self.joint = stop, iid, joint
    self.batched = chains is not None
    self.n = int(chains) if self.batched else 1
    self.seeds = seeds
    if rng is None:
      rng = 'legacy' if (not self.batched or seeds is not None) else 'philox'
    self.rng, self.seed, self.device = rng, seed, device
    self.thin, self.spl = int(thin), int(steps_per_launch)
    self.debug = (not self.batched) if debug is None else bool(debug)
    self.names = sp.keylist
    self.tr = None
    self.thresholds = None
    self.spec = None

  def _init_array(self):
    d, n = len(self.names), self.n
    init = {_key(k): v for k, v in (self.init or {}).items()}
    out = np.empty((n, d))
    for i, k in enumerate(self.names):
      if k not in init:
        raise ValueError('init value missing for {}'.format(k))
      out[:, i] = np.broadcast_to(np.asarray(init[k], np.float64), (n,))
    return out

  def _cycle_rf(self):
    """The RF whose conditional cycle this Gibbs run advances: the
    reference keeps RF.__cond_mod per RF, so consecutive samplers on the same
    RF continue mid-cycle (rf.py:446-452)."""
    if self.spec.get('kind') == 'linreg':
      tf = self.sp._tfun
      return self.sp._subfield(tf) or tf
    return self.sp._tran if isinstance(self.sp._tran, RF) else self.sp.roots

  def _cycle_len(self):
    if self.spec.get('kind') == 'linreg':
      return 3
    p = self.spec['proposal']
    return -(-int(self.spec['dim']) // int(p['tsteps']))

  def run(self):
    if self.tr is not None:
      return self
    self.spec = self.sp.lower(self.extra, self.iid, self.joint)
    self.pscale = self.spec['pscale']
    gibbs = self.spec.get('kind') == 'linreg' or \
        self.spec['proposal']['kind'] == 'gibbs'
    rf = self._cycle_rf() if gibbs else None
    self.step0 = getattr(rf, '_pbh_cond_step', 0) if gibbs else 0
    if self.spec.get('kind') == 'linreg':
      self._run_linreg()
    else:
      self._run_engine()
    if gibbs:   # the RF's __cond_mod advances by one block per SP step
      rf._pbh_cond_step = (self.step0 + self.stop) % self._cycle_len()
    return self

  def _run_engine(self):
    eng = Engine(self.spec, device=self.device)
    try:
      eng.init_chains(self._init_array())
      if self.step0:
        eng.set_step(self.step0)
      if self.rng == 'legacy':
        seeds = None if self.seeds is None else np.asarray(self.seeds)
        if seeds is None and self.batched:
          raise ValueError("rng='legacy' with chains=N needs seeds=[...]")
        eng.set_rng('replay')
        if seeds is None:
          # one chain on NumPy's GLOBAL stream: drawn on the host so that the
          # global state advances exactly as the reference leaves it
          streams = replay.legacy_streams(self.spec, self.stop, seeds,
                                          step0=self.step0)
          eng.upload_replay(streams)
          th = streams[:, -1, :] if self.spec['proposal']['kind'] != 'gibbs' \
              else None
        else:
          # RandomState(seeds[c]) per chain, generated on the device
          eng.seed_legacy(seeds)
          eng.legacy_replay(self.stop)
          th = eng.get_replay(0, self.stop, eng.stream_width() - 1) \
              if self.spec['proposal']['kind'] != 'gibbs' else None
        if th is not None:
          self.thresholds = th.T[:, self.thin - 1::self.thin]
      else:
        eng.set_rng(self.rng, self.seed)
      eng.alloc_trace(self.stop // self.thin, self.thin, debug=self.debug)
      eng.run(self.stop, steps_per_launch=self.spl)
      self.tr = eng.trace()
      self.moments = eng.moments()
    finally:
      eng.close()

  def _run_linreg(self):
    from probayes_amd import linreg
    sp = self.spec
    if self.thin != 1:
      raise L.NotLowerable('linreg Gibbs records every step (thin=1)')
    rand, rng = None, self.rng
    n_obs = len(sp['x_obs'])
    if rng == 'legacy':
      if self.batched and self.seeds is None:
        raise ValueError("rng='legacy' with chains=N needs seeds=[...]")
      rand = linreg.legacy_streams(self.stop, n_obs, sp['hyper'][4],
                                   None if self.seeds is None else self.seeds,
                                   step0=self.step0)
      rng = 'replay'
    out = linreg.run(sp['x_obs'], sp['y_obs'], self._init_array(), self.stop,
                     hyper=sp['hyper'], vsets=sp['vsets'], rng=rng,
                     seed=self.seed, rand=rand, device=self.device,
                     step0=self.step0)
    vx, vp = out['v_x'], out['v_p']
    # gibbs: p = v, u = True, s = t = None (sp_utils.py:75-84)
    self.tr = {'v_x': vx, 'v_p': vp, 'p_x': vx, 'p_p': vp,
               'u': np.ones(vp.shape, np.uint8)}
    self.moments = None

  def __iter__(self):
    self.run()
    for t in range(self.tr['v_x'].shape[1]):
      yield Step(self, t)

  def summary(self, idx=None):
    self.run()
    T = self.tr['v_x'].shape[1]
    idx = np.arange(T) if idx is None else np.asarray(idx)
    sel = (lambda a: a[0, idx]) if not self.batched else \
        (lambda a: np.moveaxis(a[:, idx], 0, 1))

    def pd(xkey, pkey):
      if xkey not in self.tr:
        return None
      xs = self.tr[xkey]
      vals = {k: sel(xs[..., i]) for i, k in enumerate(self.names)}
      return PD('p', vals, prob=sel(self.tr[pkey]), pscale=self.pscale)

    u = sel(self.tr['u']).astype(bool)
    if self.batched:
      u = u.view(FlagArray)
    else:
      u = [True if b else None for b in u]
    s = sel(self.tr['s']) if 's' in self.tr else None
    t = None if self.thresholds is None else sel(self.thresholds)
    v = pd('v_x', 'v_p')
    o, q, r = self._oqr(idx, sel)
    return OPQRSTUV(o, pd('p_x', 'p_p'), q, r, s, t, u, v)

  def _oqr(self, idx, sel):
    """The summary's o, q and r (sp.py:160-191, sd.py:253-288): o = the
    predecessor (the last accepted state; None on step 1, so summated over
    the steps after the first), q = the transition PD over (x', x) with the
    tran's value as prob, r = the reverse PD over (x, x') for an asymmetric
    tran, whose value equals q's (rf.py:536, App. A-6).  q and r need the
    recorded proposals (debug traces; single-chain samplers record them) and
    are None for Gibbs."""
    tr, names = self.tr, self.names
    if self.spec.get('kind') == 'linreg' or self.spec['scores'] == 'gibbs':
      return None, None, None
    vx, vp = tr['v_x'], tr['v_p']                 # [N, T, d], [N, T]
    later = idx[idx > 0]
    o = None
    if later.size:
      sel_o = (lambda a: a[0, later - 1]) if not self.batched else \
          (lambda a: np.moveaxis(a[:, later - 1], 0, 1))
      o = PD('p', {k: sel_o(vx[..., i]) for i, k in enumerate(names)},
             prob=sel_o(vp), pscale=self.pscale)
    if 'p_x' not in tr:
      return o, None, None
    init = self._init_array()                      # [N, d]
    prev = np.concatenate([init[:, None, :], vx[:, :-1, :]], axis=1)
    px = tr['p_x']
    tran = self.spec['tran']
    if self.spec['scores'] == 'metropolis' and self.sp._tran_spec() is None:
      qv = None
    elif tran['kind'] == 'const':
      qv = np.full(vp.shape, float(tran['value']))
    else:   # prod over the tran's order of norm.pdf(x', x + offset, scale)
      qv = None
      for k in tran['order']:
        term = scipy.stats.norm.pdf(px[..., k], loc=prev[..., k] + tran['offset'][k],
                                    scale=tran['scale'])
        qv = term if qv is None else qv * term
    succ = {k + "'": sel(px[..., i]) for i, k in enumerate(names)}
    pred = {k: sel(prev[..., i]) for i, k in enumerate(names)}
    qprob = None if qv is None else sel(qv)
    q = PD('q', dict(succ, **pred), prob=qprob, pscale=self.pscale)
    r = None
    if not tran.get('sym', True):
      r = PD('r', dict(pred, **succ), prob=qprob, pscale=self.pscale)
    return o, q, r
