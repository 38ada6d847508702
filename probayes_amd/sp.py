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
import weakref
import warnings

import numpy as np
import scipy.stats

from probayes_amd import linreg
from probayes_amd import lower as L
from probayes_amd import replay
from probayes_amd.engine import Engine
from probayes_amd.pd import PD
from probayes_amd.pscales import is_log
from probayes_amd.rv import RF, RV

MCMC_SAMPLERS = ('metropolis', 'hastings', 'gibbs')   # sp_utils.py:87-91


def _registry_kind(fn, slot):
  """The sampler name of one of the reference registry's own functions
  (sp_utils.py:19-85: <name>_scores / _thresh / _update, slot 0 / 1 / 2)
  passed as an object, identified by its module (exactly probayes.sp_utils:
  a user's own module of that name holds other semantics) and name; None for
  any other callable."""
  name = getattr(fn, '__name__', None)
  mod = getattr(fn, '__module__', None)
  if not callable(fn) or mod != 'probayes.sp_utils' or not isinstance(name, str):
    return None
  kind, _, part = name.partition('_')
  if kind in MCMC_SAMPLERS and part == ('scores', 'thresh', 'update')[slot]:
    return kind
  return None


def _no_spec_args(name, args, kwds):
  """sp.py:62-63, 79-80, 96-97: a registry name takes no arguments."""
  assert not args and not kwds, \
      "Neither args nor kwds permitted with spec '{}'".format(name)


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
    self._scores_fn = False    # scores given as the registry's function object
    self._scores_pscale = None   # ... and the pscale keyword it was given
    self._samplers = self._counter = self._last = None   # sp.py:113-128

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
    """sp.py:57-67: a registry name sets the scores and, through set_thresh,
    thresh and update too, overwriting any earlier ones (sp.py:64-65, 81-82);
    None clears the scores only.  Any other callable is wrapped as an
    Expression with the given arguments -- here only the registry's own
    scores functions, passed as objects, lower (as their name, without the
    cascade), with pscale given as a keyword (checked at lowering); other
    arguments change what the function computes and raise NotLowerable."""
    self._scores_fn, self._scores_pscale = False, None
    if scores is None:
      self._scores = None
      return
    if isinstance(scores, str) and scores in MCMC_SAMPLERS:
      _no_spec_args(scores, args, kwds)
      self._scores = scores
      self.set_thresh(scores)
      return
    kind = _registry_kind(scores, 0)
    if kind is None:
      raise L.NotLowerable('custom scores callables have no kernel')
    if kind != 'gibbs' and (args or set(kwds) - {'pscale'}):
      raise L.NotLowerable(
          '{}_scores with arguments {!r} {!r}: only the pscale keyword has a '
          'kernel form'.format(kind, args, kwds))
    self._scores, self._scores_fn = kind, True
    self._scores_pscale = kwds.get('pscale')

  def set_thresh(self, thresh=None, *args, **kwds):
    """sp.py:74-84: a registry name also sets update (overwriting it)."""
    if thresh is None:
      self._thresh = None
      return
    if isinstance(thresh, str) and thresh in MCMC_SAMPLERS:
      _no_spec_args(thresh, args, kwds)
      self._thresh = thresh
      self.set_update(thresh)
      return
    kind = _registry_kind(thresh, 1)
    if kind is None:
      raise L.NotLowerable('custom thresh callables have no kernel')
    if kind != 'gibbs' and (args or kwds):
      # metropolis_thresh(*args) is np.random.uniform(*args): other limits
      raise L.NotLowerable(
          '{}_thresh with arguments {!r} {!r} draws np.random.uniform({}) '
          '(sp_utils.py:30-31): the kernels draw U(0, 1)'.format(
              kind, args, kwds, ', '.join(map(repr, args))))
    self._thresh = kind

  def set_update(self, update=None, *args, **kwds):
    """sp.py:91-100."""
    if update is None:
      self._update = None
      return
    if isinstance(update, str) and update in MCMC_SAMPLERS:
      _no_spec_args(update, args, kwds)
      self._update = update
      return
    kind = _registry_kind(update, 2)
    if kind is None:
      raise L.NotLowerable('custom update callables have no kernel')
    if kind != 'gibbs' and (args or kwds):
      raise L.NotLowerable('{}_update takes no arguments (sp_utils.py:34-37)'
                           .format(kind))
    self._update = kind

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
    if self._scores_fn:
      # the function object sets neither thresh nor update (sp.py:57-67)
      if self._thresh is None or self._update is None:
        raise L.NotLowerable('scores given as a function set no thresh / '
                             'update: set_thresh() and set_update() too')
      # it scores with the pscale it was given: None is 1 (pscales.py:27-28),
      # i.e. the stored probabilities taken as linear ones
      if scores != 'gibbs':
        sp = self._scores_pscale
        eff = 'log' if sp is not None and is_log(sp) else \
              'lin' if sp is None or sp == 1 else None
        if eff != pscale:
          raise L.NotLowerable(
              'scores given as a function with pscale={!r} divide the {}-scaled '
              'probabilities as {} ones (div_prob, pscales.py:219-236): no '
              'kernel form'.format(sp, pscale, eff or sp))
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

  # ---- sampler registry (sp.py:113-128, 201-258) --------------------------
  def reset(self, sampler_id=None, reset_last=True):
    """sp.py:113-128: with no sampler, empties the registry; otherwise the
    sampler's counter goes to 0 and, with reset_last, its last state is
    dropped, so that its next step restarts the chains at the sampler's
    init (step 1 again: auto-accept).  reset_last=False keeps the chains
    where the last step handed out left them."""
    if self._samplers is None or sampler_id is None:
      self._samplers = []
    if self._counter is None:
      self._counter = _WeakCounter()
    if self._last is None:
      self._last = _LastStates()
    if sampler_id is None:
      return None
    sampler = self.get_sampler(sampler_id)
    self._counter[sampler] = 0
    sampler._reset(reset_last)
    if sampler not in self._last or reset_last:
      self._last[sampler] = None
    return self._samplers, self._counter, self._last

  def get_sampler(self, sampler_id=None):
    """sp.py:201-206: a sampler by index, or the sampler itself."""
    if sampler_id is None:
      return self._samplers
    if type(sampler_id) is int:
      return self._samplers[sampler_id]
    return sampler_id

  def get_counter(self, sampler_id=None):
    """sp.py:208-212: SP steps handed out since the sampler's last reset."""
    if sampler_id is None:
      return self._counter
    return self._counter[self.get_sampler(sampler_id)]

  def get_last(self, sampler_id=None):
    """sp.py:214-218: the state the sampler's next step proposes from, as an
    opqr whose p is the chains' current state (None before the first step
    and after a reset that dropped it)."""
    if sampler_id is None:
      return self._last
    return self._last[self.get_sampler(sampler_id)]

  def next(self, sampler_id, *args, **kwds):
    """sp.py:221-258: one SP step of the sampler (a Step with the
    reference's opqrstuv fields).  The sampler keeps its own init, extra
    and options; args / kwds are accepted for the reference's signature."""
    sampler = self.get_sampler(sampler_id)
    if self._counter is None:
      self.reset()
    step = sampler._next_step()
    self._counter.add(sampler, sampler.thin)
    self._last.put(sampler, step)   # OPQR(None, step.v, None, None) when read
    return step

  # ---- sampling (sp.py:261-295) ---------------------------------------------
  def sampler(self, *args, stop=None, iid=False, joint=False, chains=None,
              seeds=None, rng=None, seed=0, device=0, thin=1,
              steps_per_launch=0, debug=None, chunk=None):
    """sp.py:261-278.  stop=n: a bounded generator of n steps (the first
    step computes all n in one engine run); stop=None: unbounded, computed
    in chunks of `chunk` steps (default 256) as they are consumed.  A
    single positional int is the stop, as in the reference."""
    if self._samplers is None:
      self.reset()
    if len(args) == 1 and type(args[0]) is int and stop is None:
      stop, args = args[0], ()
    init = args[0] if args else None
    extra = args[1] if len(args) > 1 else None
    sm = Sampler(self, len(self._samplers), init, extra,
                 None if stop is None else int(stop), iid, joint, chains,
                 seeds, rng, seed, device, thin, steps_per_launch, debug, chunk)
    self._samplers.append(sm)
    self._counter[sm] = 0
    self._last[sm] = None
    return sm

  def walk(self, sampler, stop=None):
    """sp.py:281-295 (the check after each sample: a walk cut at `stop`
    draws stop + 1 steps from the sampler, as the reference's does)."""
    if stop is None and sampler.stop is None:
      warnings.warn(
          "No stop specification set - this walk may proceed indefinitely")
    steps = collections.deque()
    if stop is None and isinstance(sampler, Sampler):
      # nothing runs between the steps of this loop: the rest of each
      # computed block is handed out at once (the same Steps, counters, last
      # state and hand-out position as one next() per step)
      while True:
        bulk = sampler._bulk_steps()
        if bulk:
          steps.extend(bulk)
          continue
        try:
          steps.append(next(sampler))
        except StopIteration:
          return steps
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
    if any(s.sampler is not sm for s in samples):
      raise AssertionError('Sample must be outputted from sampler: {}'.format(sm))
    summary = sm.summary(samples)
    if conditionalise:
      for key in ('o', 'p', 'v'):
        pd = getattr(summary, key)
        if pd is not None:
          summary = summary._replace(**{key: pd.conditionalise(list(pd.keys()))})
    return summary


class _LastStates(weakref.WeakKeyDictionary):
  """SP's last states (sp.py:254-255: the last accepted opqr per sampler),
  kept as the last Step handed out and made the reference's
  OPQR(None, v, None, None) when read: handing out a step never copies a
  device-resident trace to the host."""

  def __getitem__(self, key):
    v = super().__getitem__(key)
    if isinstance(v, Step):
      v = OPQR(None, v.v, None, None)
      super().__setitem__(key, v)
    return v

  def get(self, key, default=None):
    return self[key] if key in self else default

  def put(self, key, v):
    """self[key] = v through a registered sampler's own weak reference."""
    r = getattr(key, '_ref', None)
    if r is not None and r in self.data:
      self.data[r] = v
    else:
      self[key] = v

  def values(self):
    return [self[k] for k in list(self.keys())]

  def items(self):
    return [(k, self[k]) for k in list(self.keys())]


class _WeakCounter(weakref.WeakKeyDictionary):
  """SP's step counters (sp.py:113-128: a collections.Counter keyed by
  sampler) without keeping the samplers alive: a sampler dropped by the
  caller and by SP.reset()'s registry is collected, and with it its engine's
  device buffers.  Missing samplers count 0, as in a Counter."""

  def __getitem__(self, key):
    r = getattr(key, '_ref', None)
    return self.data.get(r if r is not None else weakref.ref(key), 0)

  def add(self, key, k):
    """counter[key] += k; a registered sampler's own weak reference finds
    its entry (no new weakref per step: ~0.3 us of each handed-out step)."""
    r = getattr(key, '_ref', None)
    if r is not None and r in self.data:
      self.data[r] += k
    else:
      self[key] = self[key] + k


OPQRSTUV = collections.namedtuple('opqrstuv', ['o', 'p', 'q', 'r', 's', 't',
                                                'u', 'v'])
OPQR = collections.namedtuple('opqr', ['o', 'p', 'q', 'r'])


class _DeviceTrace:
  """A block's trace arrays (v_x [N, T, d], v_p [N, T], u [N, T]; debug
  p_x, p_p, s) left in the engine's device trace until first read: a
  sampler's steps are handed out without copying T x N x (8d + 9) bytes to
  the host, and a caller who reduces on the device or reads a few steps never
  pays for the rest.  The sampler copies it (materialize) before anything
  reuses the engine's trace."""

  __slots__ = ('_eng', '_keys', '_data')

  def __init__(self, eng, debug):
    self._eng = eng
    self._keys = ('v_x', 'v_p', 'u') + (('p_x', 'p_p', 's') if debug else ())
    self._data = None

  def materialize(self):
    if self._data is None:
      self._data = self._eng.trace()
      self._eng = None
    return self._data

  def __getitem__(self, key):
    return self.materialize()[key]

  def get(self, key, default=None):
    return self[key] if key in self._keys else default

  def __contains__(self, key):
    return key in self._keys

  def keys(self):
    return self._keys


class _LazyPrev:
  """A block's last record (x [N, d], lp [N]) as the next block's
  predecessor state, read when that block is computed -- after _settle has
  copied the block to the host."""

  __slots__ = ('block',)

  def __init__(self, block):
    self.block = block

  def __iter__(self):
    tr = self.block.tr
    return iter((np.array(tr['v_x'][:, -1, :]), np.array(tr['v_p'][:, -1])))


class _Block:
  """Records [0, T) of one engine run of a sampler: trace arrays tr (v_x
  [N, T, d], v_p [N, T], u [N, T]; debug p_x, p_p, s; a dict or a
  _DeviceTrace), thresholds [N, T] or None (or a function that copies them
  from the engine's replay rows), the state before record 0 (prev_x [N, d],
  prev_p [N]), whether record 0 is step 1 of a sampler epoch (first: no
  predecessor), the global step of its first step (g0), and what a rewind
  into it needs (rewind)."""

  __slots__ = ('tr', '_thr', '_thr_fn', 'prev_x', 'prev_p', 'first', 'g0', 'T',
               'rewind')

  def __init__(self, tr, thr, prev_x, prev_p, first, g0, rewind, T=None):
    self.tr, self.prev_x, self.prev_p = tr, prev_x, prev_p
    self._thr, self._thr_fn = (None, thr) if callable(thr) else (thr, None)
    self.first, self.g0, self.rewind = first, g0, rewind
    self.T = tr['v_x'].shape[1] if T is None else T

  @property
  def thr(self):
    if self._thr_fn is not None:
      self._thr, self._thr_fn = self._thr_fn(), None
    return self._thr

  def materialize(self):
    """Copies whatever still sits in the engine (before it is reused)."""
    if isinstance(self.tr, _DeviceTrace):
      self.tr.materialize()
    _ = self.thr


class Step:
  """One recorded step of a Sampler; fields as the reference's opqrstuv
  (sp.py:257-258), built lazily from its block's trace arrays."""

  __slots__ = ('sampler', 'block', 'j')

  def __init__(self, sampler, block, j):
    self.sampler, self.block, self.j = sampler, block, j

  def _pd(self, xs, ps, t):
    sm = self.sampler
    vals = {k: xs[..., t, i] if sm.batched else float(xs[0, t, i])
            for i, k in enumerate(sm.names)}
    prob = ps[..., t] if sm.batched else float(ps[0, t])
    return PD('p', vals, prob=prob, pscale=sm.pscale)

  @property
  def v(self):
    return self._pd(self.block.tr['v_x'], self.block.tr['v_p'], self.j)

  @property
  def p(self):
    tr = self.block.tr
    if 'p_x' not in tr:
      return None
    return self._pd(tr['p_x'], tr['p_p'], self.j)

  @property
  def o(self):
    b, j = self.block, self.j
    if j > 0:
      return self._pd(b.tr['v_x'], b.tr['v_p'], j - 1)
    if b.first:
      return None
    return self._pd(b.prev_x[:, None, :], b.prev_p[:, None], 0)

  @property
  def u(self):
    u = self.block.tr['u'][:, self.j].astype(bool)
    if self.sampler.batched:
      return u
    return True if u[0] else None

  @property
  def s(self):
    tr = self.block.tr
    if 's' not in tr:
      return None
    v = tr['s'][:, self.j]
    if self.sampler.batched:
      return v
    return None if np.isnan(v[0]) else float(v[0])

  @property
  def t(self):
    th = self.block.thr
    if th is None:
      return None
    return th[:, self.j] if self.sampler.batched else float(th[0, self.j])

  def astuple(self):
    return OPQRSTUV(self.o, self.p, None, None, self.s, self.t, self.u, self.v)

  def __getitem__(self, i):
    return self.astuple()[i]


class _GlobalStream:
  """Draws the single-chain legacy stream from NumPy's GLOBAL RandomState
  ahead of use and keeps the global state exactly where the reference
  leaves it: states[k] is the global state after step k's draws; handing
  out step k sets it, and a draw made by anyone else in between (the global
  state is not states[k - 1] any more) invalidates the steps drawn ahead."""

  @staticmethod
  def state():
    return np.random.get_state()

  @staticmethod
  def same(a, b):
    return a[2:] == b[2:] and np.array_equal(a[1], b[1])


class Sampler:
  """A lowered, batched MH/Gibbs process (sp.py:261-278, sp_utils.py:8-16):
  an iterator of Steps.  Steps are computed by the engine in blocks (all of
  a bounded sampler's steps at once, `chunk` steps at a time when
  unbounded) and handed out one at a time; SP.reset / SP.next / get_last /
  get_counter act on the steps handed out, rewinding the engine when it ran
  ahead of them (the counter-based production RNG and the device legacy
  streams continue exactly as an uninterrupted run would)."""

  def __init__(self, sp, sid, init, extra, stop, iid, joint, chains, seeds,
               rng, seed, device, thin, steps_per_launch, debug, chunk):
    self.sp, self.sid, self.init, self.extra = sp, sid, init, extra
    self.stop, self.iid, self.joint = stop, iid, joint
    self.batched = chains is not None
    self.n = int(chains) if self.batched else 1
    self.seeds = seeds
    if rng is None:
      rng = 'legacy' if (not self.batched or seeds is not None) else 'philox'
    self.rng, self.seed, self.device = rng, seed, device
    self.thin, self.spl = int(thin), int(steps_per_launch)
    self.chunk = int(chunk) if chunk else 256
    if self.chunk % self.thin:
      self.chunk += self.thin - self.chunk % self.thin
    self.debug = (not self.batched) if debug is None else bool(debug)
    self.names = sp.keylist
    self.spec = None
    self._eng = None        # the engine (MH / CondCov Gibbs)
    self._lx = None         # linreg: the chains' state [N, 3] (host)
    self._rs = None         # linreg legacy streams: an Engine of device RandomStates
    self._g = 0             # global step of the next step to compute
    self._cur = None        # block being handed out and its next record
    self._j = 0
    self._handed = None     # (block, j) of the last record handed out
    self._epoch = True      # the next step starts an epoch (at init)
    self._drawn = []        # (global step, steps) drawn from seeded streams
    self._done = False      # a bounded sampler ran out (sp_utils.py:14-16)
    # global-stream draw-ahead (rng 'legacy', seeds None): steps computed
    # ahead per block; back to one step after a caller's own draw forced a
    # rewind, doubled per block after that (interleaved samplers cost O(1)
    # per step instead of a redraw of the whole remaining stop)
    self._ahead = self.chunk
    self.n_computed = 0     # chain-steps' worth of steps run (diagnostic)
    self._prev = None       # the state before the next block, when known on the host
    self._ref = weakref.ref(self)   # the SP registry's key for this sampler
    self._gibbs = None      # _is_gibbs(), fixed once lowered

  def __repr__(self):
    return '<probayes_amd Sampler {} stop={}>'.format(self.sid, self.stop)

  def __hash__(self):
    return id(self)

  # ---- the generator (sp_utils.py:8-16) ------------------------------------
  def __iter__(self):
    return self

  def __next__(self):
    if self._done:
      raise StopIteration
    if self.stop is not None and self.sp.get_counter(self) >= self.stop:
      self.sp.reset(self)
      self._done = True
      raise StopIteration
    return self.sp.next(self)

  def _bulk_steps(self):
    """The steps next() would hand out from the current block, all at once,
    when no per-step work is due (not after the block's end or the stop, no
    global-stream rewind states, no Gibbs cycle phase): SP.walk's fast path.
    Returns [] when the next step needs next()."""
    cur = self._cur
    if (self._done or self._epoch or cur is None or self._gibbs is not False or
        'states' in cur.rewind or self._j >= cur.T):
      return []
    k = cur.T - self._j
    if self.stop is not None:
      k = min(k, (self.stop - self.sp.get_counter(self)) // self.thin)
    if k <= 0:
      return []
    j0 = self._j
    out = [Step(self, cur, j) for j in range(j0, j0 + k)]
    self._j = j0 + k
    self._handed = (cur, j0 + k - 1)
    self.sp._counter.add(self, k * self.thin)
    self.sp._last.put(self, out[-1])
    return out

  # ---- set-up ------------------------------------------------------------
  def _init_array(self):
    d, n = len(self.names), self.n
    init = {_key(k): v for k, v in (self.init or {}).items()}
    out = np.empty((n, d))
    vals = []
    for k in self.names:
      if k not in init:
        raise ValueError('init value missing for {}'.format(k))
      vals.append(np.asarray(init[k], np.float64))
    if all(v.size == 1 for v in vals):   # one row for every chain: a contiguous fill
      out[:] = np.array([float(v.reshape(-1)[0]) for v in vals])
      return out
    for i, v in enumerate(vals):
      out[:, i] = np.broadcast_to(v, (n,))
    return out

  def _is_gibbs(self):
    return self.spec.get('kind') == 'linreg' or \
        self.spec['proposal']['kind'] == 'gibbs'

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

  def _lower(self):
    if self.spec is not None:
      return
    self.spec = self.sp.lower(self.extra, self.iid, self.joint)
    self.pscale = self.spec['pscale']
    self._gibbs = self._is_gibbs()
    if self.rng == 'legacy' and self.batched and self.seeds is None:
      raise ValueError("rng='legacy' with chains=N needs seeds=[...]")
    if self.spec.get('kind') == 'linreg' and self.thin != 1:
      raise L.NotLowerable('linreg Gibbs records every step (thin=1)')

  def _start_epoch(self):
    """Chains back at init, step 1 next (auto-accept); a Gibbs cycle starts
    at its RF's phase; every generator continues."""
    self._settle()
    gibbs = self._is_gibbs()
    phase = getattr(self._cycle_rf(), '_pbh_cond_step', 0) if gibbs else 0
    g = self._g
    if gibbs:   # the next step index at the RF's cycle phase
      g += (phase - g) % self._cycle_len()
    init = self._init_array()
    if self.spec.get('kind') == 'linreg':
      self._lx = init
      if self.rng == 'legacy' and self.seeds is not None and self._rs is None:
        self._rs = self._linreg_streams()
    elif self._eng is None:
      eng = Engine(self.spec, device=self.device)
      self._eng = eng
      eng.init_chains(init)
      if g:
        eng.set_step(g)
      if self.rng == 'legacy':
        eng.set_rng('replay')
        if self.seeds is not None:
          # RandomState(seeds[c]) per chain, generated on the device; the MH
          # thresholds kept for the steps' t
          eng.seed_legacy(np.asarray(self.seeds))
          if self.spec['proposal']['kind'] != 'gibbs':
            eng.set_record_threshold(True)
      else:
        eng.set_rng(self.rng, self.seed)
    else:
      self._eng.set_chains(init, np.zeros(self.n), g, False)
    self._g = g
    self._epoch_first = True
    # the state before the epoch's first step: init, lp 0 (as init_chains /
    # set_chains leave it)
    self._prev = (init, np.zeros(self.n))

  def close(self):
    """Frees the engine (also done when the sampler is collected)."""
    if self._rs is not None:   # the linreg chains' device RandomStates
      self._rs.close()
      self._rs = None
    if self._eng is not None:
      try:
        self._settle()   # steps handed out keep their data
      except Exception:   # a failed engine: nothing to copy
        pass
      self._eng.close()
      self._eng = None

  def __del__(self):
    try:
      self.close()
    except Exception:   # interpreter shutdown
      pass

  # ---- computing blocks ----------------------------------------------------
  def _global_stream(self):
    return self.rng == 'legacy' and self.seeds is None

  def _block_steps(self):
    k = self.chunk
    if self.stop is not None:
      left = self.stop - self.sp.get_counter(self)
      if left > 0:
        k = left - left % self.thin if left >= self.thin else self.thin
    if self._global_stream():
      k = min(k, self._ahead)
    return k

  def _draw_global(self, k):
    """k steps of the single chain's legacy stream from NumPy's global
    state, with the global state after each step."""
    out, states = [], []
    for t in range(k):
      if self.spec.get('kind') == 'linreg':
        out.append(linreg.legacy_streams(1, len(self.spec['x_obs']),
                                         self.spec['hyper'][4], None,
                                         step0=self._g + t))
      else:
        out.append(replay.legacy_streams(self.spec, 1, None,
                                         step0=self._g + t))
      states.append(_GlobalStream.state())
    return np.concatenate(out, axis=0), states

  def _settle(self):
    """Copies the current block's data still held by the engine (its trace,
    its replay rows) before the engine runs, rewinds or reseeds again."""
    if self._cur is not None:
      self._cur.materialize()

  def _compute(self):
    """Runs the next block from the current chain state."""
    self._settle()
    k = self._block_steps()
    first = self._epoch_first
    self._epoch_first = False
    g0 = self._g
    rewind = {}
    if self.spec.get('kind') == 'linreg':
      tr, thr, prev_x, prev_p = self._compute_linreg(k, rewind)
    else:
      tr, thr, prev_x, prev_p = self._compute_engine(k, rewind)
    self._g = g0 + k
    self.n_computed += k
    if self._global_stream():
      self._ahead = min(2 * self._ahead, 1 << 30)
    # Steps keep their own block; the sampler keeps only the current one
    self._cur, self._j = _Block(tr, thr, prev_x, prev_p, first, g0, rewind,
                                T=k // self.thin), 0
    # the next block's predecessor state: this block's last record (read
    # from the host copy _settle makes before that block runs)
    cur = self._cur
    self._prev = None if self._is_gibbs() else _LazyPrev(cur)   # (MH: lp = v.prob)

  def _compute_engine(self, k, rewind):
    eng = self._eng
    if self._prev is not None:   # known on the host: no device copy
      prev_x, prev_p = tuple(self._prev)
    else:
      prev_x, prev_p = eng.state()
    thr = None
    if self.rng == 'legacy':
      if self.seeds is None:
        streams, rewind['states'] = self._draw_global(k)
        eng.upload_replay(streams)
        thr = streams[:, -1, :] if self.spec['proposal']['kind'] != 'gibbs' else None
      else:
        # the device RandomStates drawn inside the REPLAY steps (the fused
        # kernel, pbh_legacy_run); the thresholds stay on the device until a
        # step's t or the summary reads them
        self._drawn.append((self._g, k))   # steps drawn since seeding
        # (the run writes every record: no zero fill)
        eng.alloc_trace(k // self.thin, self.thin, debug=self.debug, fill=False)
        eng.legacy_run(k, steps_per_launch=self.spl)
        if self.spec['proposal']['kind'] != 'gibbs':
          thin = self.thin
          thr = lambda: eng.get_thresholds(0, k).T[:, thin - 1::thin]
        return _DeviceTrace(eng, self.debug), thr, prev_x, prev_p
      if isinstance(thr, np.ndarray):
        thr = thr.T[:, self.thin - 1::self.thin]
    elif self.rng == 'xoshiro':
      rewind['ck'] = eng.checkpoint()     # the generators at block start
    eng.alloc_trace(k // self.thin, self.thin, debug=self.debug, fill=False)
    eng.run(k, steps_per_launch=self.spl)
    return _DeviceTrace(eng, self.debug), thr, prev_x, prev_p

  def _compute_linreg(self, k, rewind):
    sp = self.spec
    rand, rng = None, self.rng
    if rng == 'legacy':
      if self.seeds is None:
        rand, rewind['states'] = self._draw_global(k)
      else:
        rand = self._linreg_draws(self._g, k)
        self._drawn.append((self._g, k))
      rng = 'replay'
    prev_x = self._lx
    out = linreg.run(sp['x_obs'], sp['y_obs'], self._lx, k, hyper=sp['hyper'],
                     vsets=sp['vsets'], rng=rng, seed=self.seed, rand=rand,
                     device=self.device, step0=self._g)
    vx, vp = out['v_x'], out['v_p']
    self._lx = out['final_x']
    # gibbs: p = v, u = True, s = t = None (sp_utils.py:75-84)
    tr = {'v_x': vx, 'v_p': vp, 'p_x': vx, 'p_p': vp,
          'u': np.ones(vp.shape, np.uint8)}
    return tr, None, prev_x, np.full(self.n, np.nan)

  def _linreg_draws(self, g, k, keep=True):
    """k steps from the seeded per-chain RandomStates (linreg's legacy
    order: standard_gamma on y_sigma steps, gauss otherwise), drawn on the
    device (pbh_legacy_draws: one NumPy RandomState per chain, NumPy's
    legacy_standard_gamma): [k, N]."""
    alpha = self.spec['hyper'][4] + 0.5 * len(self.spec['x_obs'])
    return self._rs.legacy_draws(k, g, 'linreg', alpha)

  def _linreg_streams(self):
    """The seeded linreg chains' RandomStates on the device: an engine
    that holds only the legacy generators (pbh_legacy_seed)."""
    from probayes_amd.spec import make_spec
    eng = Engine(make_spec(1, target={'kind': 'diag_gauss', 'mu': np.zeros(1),
                                      'sigma': np.ones(1)},
                           proposal={'kind': 'gauss', 'loc': 0., 'scale': 1.},
                           scores='hastings', pscale='log',
                           tran={'kind': 'const', 'value': 1.0, 'sym': True}),
                 device=self.device)
    eng.init_chains(np.zeros((self.n, 1)))
    eng.seed_legacy(np.asarray(self.seeds))
    return eng

  def _reseed_streams(self, keep):
    """Rewinds the seeded legacy streams to the draws of the first `keep`
    steps since seeding: seed again, then draw and discard those steps at
    their global step indices (the draw kinds and counts of a Gibbs step
    follow its place in the cycle)."""
    log, self._drawn = self._drawn, []
    linreg_ = self.spec.get('kind') == 'linreg'
    if linreg_:
      self._rs.seed_legacy(np.asarray(self.seeds))
    else:
      eng = self._eng
      eng.seed_legacy(np.asarray(self.seeds))
      x, p = eng.state()
    for g, k in log:
      k = min(k, keep)
      for b in range(0, k, 256):
        m = min(256, k - b)
        if linreg_:
          self._linreg_draws(g + b, m)
        else:
          eng.set_chains(x, p, g + b, True)
          eng.legacy_replay(m)
      if k:
        self._drawn.append((g, k))
      keep -= k

  # ---- handing out steps ---------------------------------------------------
  def _next_step(self):
    self._lower()
    if self._epoch:
      self._start_epoch()
      self._epoch = False
      self._cur = None
    cur = self._cur
    if cur is not None and self._j < cur.T and 'states' in cur.rewind and \
        self._j > 0 and not _GlobalStream.same(
            _GlobalStream.state(), cur.rewind['states'][self._j * self.thin - 1]):
      # someone drew from the global stream since the last step: the steps
      # drawn ahead are not the reference's any more
      self._rewind_to_handed()
      self._ahead = self.thin
      cur = None
    if cur is None or self._j >= cur.T:
      self._compute()
      cur = self._cur
    j = self._j
    self._j += 1
    if 'states' in cur.rewind:
      np.random.set_state(cur.rewind['states'][(j + 1) * self.thin - 1])
      if self._j >= cur.T:   # fully handed out: no rewind into it any more
        del cur.rewind['states']
    self._handed = (cur, j)
    if self._gibbs:   # the RF's __cond_mod follows the steps handed out
      self._cycle_rf()._pbh_cond_step = \
          (cur.g0 + (j + 1) * self.thin) % self._cycle_len()
    return Step(self, cur, j)

  def _rewind_to_handed(self):
    """Puts the chains (and their generators) where the last step handed
    out left them: the engine may have run ahead of it."""
    self._settle()
    cur = self._cur
    if cur is None or self._j >= cur.T:
      return   # nothing ahead
    b, j = self._handed if self._handed is not None else (cur, -1)
    if b is not cur:
      return
    g = cur.g0 + (j + 1) * self.thin
    x = cur.prev_x if j < 0 else cur.tr['v_x'][:, j, :]
    p = cur.prev_p if j < 0 else cur.tr['v_p'][:, j]
    has_pred = not (j < 0 and cur.first)
    seeded = self.rng == 'legacy' and self.seeds is not None
    if seeded:   # the streams: what was drawn before this block + j + 1 steps
      total = sum(k for _, k in self._drawn)
      self._reseed_streams(total - cur.T * self.thin + (j + 1) * self.thin)
    if self.spec.get('kind') == 'linreg':
      self._lx = np.array(x)
    elif 'ck' in cur.rewind:
      # xoshiro: back to the block start, then the handed steps again (the
      # same draws, the same chains)
      eng = self._eng
      eng.restore(cur.rewind['ck'])
      if j >= 0:
        eng.run((j + 1) * self.thin, steps_per_launch=self.spl)
    else:
      # counter-based draws (Philox) or host streams: the state is all; the
      # global NumPy state was set when step j was handed out and any draw
      # made since then is the user's own, which the reference would see too
      self._eng.set_chains(x, p, g, has_pred)
    self._g = g
    self._epoch_first = j < 0 and cur.first
    self._cur, self._j = None, 0
    self._prev = None   # the engine holds the rewound state

  def _reset(self, reset_last):
    """SP.reset: reset_last restarts the chains at init at the next step;
    otherwise they continue from the last step handed out."""
    if reset_last:
      self._epoch = True
    else:
      self._rewind_to_handed()
    self._cur, self._j = None, 0

  # ---- summaries -------------------------------------------------------------
  @staticmethod
  def _runs(steps):
    """(block, record indices) per run of consecutive steps from one block."""
    i = 0
    while i < len(steps):
      b = steps[i].block
      k = i
      while k < len(steps) and steps[k].block is b:
        k += 1
      yield b, np.array([s.j for s in steps[i:k]])
      i = k

  @staticmethod
  def _span(js):
    """js as a slice when it is a contiguous ascending range (a walk's steps
    are): the summary then holds views of the host trace, not copies."""
    if len(js) and js[-1] - js[0] + 1 == len(js) and np.all(np.diff(js) == 1):
      return slice(int(js[0]), int(js[-1]) + 1)
    return js

  def _gather(self, steps, get):
    """[N, len(steps), ...] from get(block) [N, T, ...] at the steps'
    records: a view for one contiguous run (a whole walk of one block), one
    index per run of steps from the same block otherwise."""
    parts = []
    for b, js in self._runs(steps):
      a = get(b)
      if a is None:
        return None
      parts.append(a[:, self._span(js)])
    if len(parts) == 1:
      return parts[0]
    return np.concatenate(parts, axis=1)

  def _gather_prev(self, steps, key):
    """The state before each step (its predecessor record, or the block's
    prev for a block's record 0): key 'x' -> [N, len, d], 'p' -> [N, len];
    a view of the records when no step is a block's record 0."""
    parts = []
    for b, js in self._runs(steps):
      a = b.tr['v_' + key]
      sp = self._span(js)
      if isinstance(sp, slice) and sp.start >= 1:
        parts.append(a[:, sp.start - 1:sp.stop - 1])
        continue
      prev = b.prev_x[:, None, :] if key == 'x' else b.prev_p[:, None]
      parts.append(np.concatenate([prev, a[:, :-1]], 1)[:, js])
    if len(parts) == 1:
      return parts[0]
    return np.concatenate(parts, axis=1)

  def summary(self, steps):
    steps = list(steps)
    sel = (lambda a: a[0]) if not self.batched else (lambda a: np.moveaxis(a, 0, 1))
    tr = lambda key: (lambda b: b.tr.get(key))

    def pd(xkey, pkey, subset=None):
      xs = self._gather(steps if subset is None else subset, tr(xkey))
      if xs is None:
        return None
      ps = self._gather(steps if subset is None else subset, tr(pkey))
      vals = {k: sel(xs[..., i]) for i, k in enumerate(self.names)}
      return PD('p', vals, prob=sel(ps), pscale=self.pscale)

    u = sel(self._gather(steps, tr('u'))).astype(bool)
    if self.batched:
      u = u.view(FlagArray)
    else:
      u = [True if b else None for b in u]
    s_ = self._gather(steps, tr('s'))
    s = None if s_ is None else sel(s_)
    t_ = self._gather(steps, lambda b: b.thr)
    t = None if t_ is None else sel(t_)
    v = pd('v_x', 'v_p')
    o, q, r = self._oqr(steps, sel)
    return OPQRSTUV(o, pd('p_x', 'p_p'), q, r, s, t, u, v)

  def _oqr(self, steps, sel):
    """The summary's o, q and r (sp.py:160-191, sd.py:253-288): o = the
    predecessor (the last accepted state; None on step 1 of an epoch, so
    summated over the other steps), q = the transition PD over (x', x) with
    the tran's value as prob, r = the reverse PD over (x, x') for an
    asymmetric tran, whose value equals q's (rf.py:536, App. A-6).  q and r
    need the recorded proposals (debug traces; single-chain samplers record
    them) and are None for Gibbs."""
    names = self.names
    if self.spec.get('kind') == 'linreg' or self.spec['scores'] == 'gibbs':
      return None, None, None
    # the state before each step: the previous record, or the block's prev
    later = [st for st in steps if not (st.j == 0 and st.block.first)]
    o = None
    if later:
      ox = self._gather_prev(later, 'x')
      op = self._gather_prev(later, 'p')
      o = PD('p', {k: sel(ox[..., i]) for i, k in enumerate(names)},
             prob=sel(op), pscale=self.pscale)
    px = self._gather(steps, lambda b: b.tr.get('p_x'))
    if px is None:
      return o, None, None
    prev = self._gather_prev(steps, 'x')
    vp = self._gather(steps, lambda b: b.tr['v_p'])
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
