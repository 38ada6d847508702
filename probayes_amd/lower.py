"""Lowering: from the SP facade's Python callables to a kernel spec.

The reference accepts arbitrary Python callables for the density, the
transition and the delta (rf.py:91,169; field.py:220).  The GPU engine
recognises a closed set of forms.  Callables are lowered
by *symbolic tracing*: they are called once with symbolic stand-ins for the
variables while scipy.stats.norm.rvs / .pdf / .logpdf and uniform.pdf are
temporarily replaced by recorders, so the recorded calls describe the
callable exactly (no random number is drawn by tracing).  A callable whose
trace is not one of the recognised forms raises NotLowerable -- there is no
CPU fallback.

Recognised forms
  delta  lambda: Delta(k1=norm.rvs(loc, scale), ...)            -> gauss
  tran   lambda **kw: c                                          -> const
         prod of norm.pdf(kw[k'], loc=kw[k] + off, scale=s)      -> gauss_pdf
  prob   sum_k norm.logpdf(kw[k], mu_k, sigma_k) (dims in order) -> diag_gauss
         prod_k uniform.pdf(kw[k], lo_k, scale_k)                -> uniform_pdf
         a = logw + sum_i norm.logpdf(kw[k_i], mu[:, i], sd) (vectors over
         components), then m = np.max(a); m + np.log(np.sum(np.exp(a - m)))
         or scipy.special.logsumexp(a)                          -> gmm
         (traced through NumPy's __array_ufunc__ / __array_function__)
  plus the scipy objects themselves (norm.pdf/logpdf, uniform.pdf,
  multivariate_normal) and the descriptor callables of probayes_amd.models.
"""
import contextlib
import numbers

import numpy as np
import scipy.stats


class NotLowerable(NotImplementedError):
  """The model form has no GPU kernel (no CPU fallback exists)."""


# ---------------------------------------------------------------------------
# symbolic values
# ---------------------------------------------------------------------------
class Sym:
  """A variable reference plus a constant offset."""

  def __init__(self, name, off=0.0):
    self.name, self.off = name, float(off)

  def __add__(self, c):
    if isinstance(c, numbers.Real):
      return Sym(self.name, self.off + float(c))
    return NotImplemented

  __radd__ = __add__

  def __sub__(self, c):
    if isinstance(c, numbers.Real):
      return Sym(self.name, self.off - float(c))
    return NotImplemented


class Draw:
  """A recorded norm.rvs(loc, scale) call."""

  def __init__(self, j, loc, scale):
    self.j, self.loc, self.scale = j, float(loc), float(scale)


class Term:
  """A recorded density call; products / sums build Expr lists."""

  def __init__(self, kind, x, loc, scale):
    self.kind, self.x, self.loc, self.scale = kind, x, loc, scale

  def __mul__(self, o):
    return Expr('prod', [self]) * o

  def __add__(self, o):
    return Expr('sum', [self]) + o

  __radd__ = None  # set below


class Expr:
  def __init__(self, op, terms):
    self.op, self.terms = op, list(terms)

  def __mul__(self, o):
    if self.op != 'prod':
      raise NotLowerable('mixed sum/product density')
    if isinstance(o, Term):
      return Expr('prod', self.terms + [o])
    if isinstance(o, Expr) and o.op == 'prod':
      return Expr('prod', self.terms + o.terms)
    raise NotLowerable('product with a non-density factor')

  def __add__(self, o):
    if self.op != 'sum':
      raise NotLowerable('mixed sum/product density')
    if isinstance(o, Term):
      return Expr('sum', self.terms + [o])
    if isinstance(o, Expr) and o.op == 'sum':
      return Expr('sum', self.terms + o.terms)
    raise NotLowerable('sum with a non-density term')

  def __radd__(self, o):
    # Python sum() starts from 0
    if isinstance(o, numbers.Real) and o == 0:
      return self
    raise NotLowerable('sum with a constant')


def _term_radd(self, o):
  if isinstance(o, numbers.Real) and o == 0:
    return Expr('sum', [self])
  raise NotLowerable('sum with a constant')


Term.__radd__ = _term_radd
Term.__rmul__ = lambda self, o: Expr('prod', [self]) * o


def _num(v, what):
  if isinstance(v, (Sym, Draw, Term, Expr)):
    raise NotLowerable('{} must be a constant'.format(what))
  return float(v)


@contextlib.contextmanager
def _patched(obj, **fns):
  saved = {k: obj.__dict__.get(k, None) for k in fns}
  try:
    for k, f in fns.items():
      setattr(obj, k, f)
    yield
  finally:
    for k, v in saved.items():
      if v is None:
        delattr(obj, k)
      else:
        setattr(obj, k, v)


def _loc_scale(args, kwds):
  loc = kwds.get('loc', args[0] if len(args) > 0 else 0.)
  scale = kwds.get('scale', args[1] if len(args) > 1 else 1.)
  return loc, scale


# ---------------------------------------------------------------------------
# delta
# ---------------------------------------------------------------------------
def trace_delta(fn, keys):
  """lambda: Delta(k=norm.rvs(loc, scale), ...) -> gauss proposal."""
  draws = []

  def rvs(*args, **kwds):
    if kwds.get('size') not in (None, ()):
      raise NotLowerable('norm.rvs with size in a delta')
    loc, scale = _loc_scale(args, kwds)
    d = Draw(len(draws), _num(loc, 'rvs loc'), _num(scale, 'rvs scale'))
    draws.append(d)
    return d

  with _patched(scipy.stats.norm, rvs=rvs):
    out = fn()
  if hasattr(out, '_asdict'):
    out = out._asdict()
  if not isinstance(out, dict):
    raise NotLowerable('delta callable must return Delta(...)')
  d = len(keys)
  loc, scale = np.zeros(d), np.ones(d)
  order = np.full(d, -1, np.int32)
  if len(draws) != d or set(out) != set(keys):
    raise NotLowerable('delta must draw exactly one norm.rvs per variable')
  for key, v in out.items():
    if not isinstance(v, Draw):
      raise NotLowerable('delta value for {} is not a norm.rvs draw'.format(key))
    k = keys.index(key)
    order[v.j] = k
    loc[k], scale[k] = v.loc, v.scale
  return {'kind': 'gauss', 'loc': loc, 'scale': scale, 'order': order}


# ---------------------------------------------------------------------------
# tran
# ---------------------------------------------------------------------------
def _norm_pdf_term(*args, **kwds):
  x = args[0] if args else kwds.pop('x')
  loc, scale = _loc_scale(args[1:], kwds)
  return Term('norm_pdf', x, loc, scale)


def trace_tran(fn, keys):
  """Returns {'kind': 'const'|'gauss_pdf', ...} (sym filled by the caller)."""
  kw = {}
  for k in keys:
    kw[k] = Sym(k)
    kw[k + "'"] = Sym(k + "'")
  with _patched(scipy.stats.norm, pdf=_norm_pdf_term):
    try:
      out = fn(**kw)
    except NotLowerable:
      raise
    except Exception as e:   # e.g. arithmetic a Sym does not support
      raise NotLowerable('tran callable not traceable: {}'.format(e))
  if isinstance(out, numbers.Real):
    return {'kind': 'const', 'value': float(out)}
  terms = [out] if isinstance(out, Term) else \
      (out.terms if isinstance(out, Expr) and out.op == 'prod' else None)
  if not terms:
    raise NotLowerable('tran must be a constant or a product of norm.pdf')
  d = len(keys)
  off = np.zeros(d)
  order = []
  scale = None
  for t in terms:
    if not (isinstance(t.x, Sym) and t.x.name.endswith("'") and t.x.off == 0
            and isinstance(t.loc, Sym) and t.loc.name + "'" == t.x.name):
      raise NotLowerable('tran term is not norm.pdf(x\', loc=x + c, scale)')
    k = keys.index(t.loc.name)
    off[k] = t.loc.off
    order.append(k)
    s = _num(t.scale, 'tran scale')
    if scale is not None and s != scale:
      raise NotLowerable('tran scales differ across variables')
    scale = s
  if sorted(order) != list(range(d)):
    raise NotLowerable('tran must cover every variable once')
  return {'kind': 'gauss_pdf', 'scale': scale, 'offset': off,
          'order': np.asarray(order, np.int32)}


# ---------------------------------------------------------------------------
# prob
# ---------------------------------------------------------------------------
def trace_prob(fn, keys):
  """User density callable -> target dict, or NotLowerable."""
  def logpdf(*args, **kwds):
    x = args[0] if args else kwds.pop('x')
    loc, scale = _loc_scale(args[1:], kwds)
    return Term('norm_logpdf', x, loc, scale)

  def updf(*args, **kwds):
    x = args[0] if args else kwds.pop('x')
    loc, scale = _loc_scale(args[1:], kwds)
    return Term('uniform_pdf', x, loc, scale)

  kw = {k: Sym(k) for k in keys}
  with _patched(scipy.stats.norm, logpdf=logpdf), \
       _patched(scipy.stats.uniform, pdf=updf):
    try:
      out = fn(**kw)
    except NotLowerable:
      raise
    except Exception as e:
      raise NotLowerable('density callable not traceable: {}'.format(e))
  terms = [out] if isinstance(out, Term) else \
      (out.terms if isinstance(out, Expr) else None)
  if not terms:
    raise NotLowerable('density is not a recognised form')
  kinds = {t.kind for t in terms}
  d = len(keys)
  for i, t in enumerate(terms):
    if not (isinstance(t.x, Sym) and t.x.off == 0 and t.x.name == keys[i]):
      raise NotLowerable('density terms must take the variables in order')
  if len(terms) != d:
    raise NotLowerable('density must have one term per variable')
  if kinds == {'norm_logpdf'} and (isinstance(out, Term) or out.op == 'sum'):
    return {'kind': 'diag_gauss',
            'mu': np.array([_num(t.loc, 'loc') for t in terms]),
            'sigma': np.array([_num(t.scale, 'scale') for t in terms])}, 'log'
  if kinds == {'uniform_pdf'} and (isinstance(out, Term) or out.op == 'prod'):
    return {'kind': 'uniform_pdf',
            'lo': np.array([_num(t.loc, 'loc') for t in terms]),
            'scale': np.array([_num(t.scale, 'scale') for t in terms])}, 'lin'
  raise NotLowerable('density is not a recognised form')


# ---------------------------------------------------------------------------
# prob: log-sum-exp mixtures, traced through NumPy's dispatch protocols
# ---------------------------------------------------------------------------
class Node:
  """A symbolic array value: NumPy ufuncs and np.max / np.sum on it build a
  graph instead of computing (NEP 13 / NEP 18 dispatch)."""
  __array_priority__ = 1000

  def __init__(self, op, *args):
    self.op, self.args = op, args

  _UFUNCS = {np.add: 'add', np.subtract: 'sub', np.exp: 'exp', np.log: 'log'}

  def __array_ufunc__(self, ufunc, method, *inputs, **kw):
    if method != '__call__' or kw or ufunc not in self._UFUNCS:
      raise NotLowerable('{}.{} in a density'.format(ufunc.__name__, method))
    return Node(self._UFUNCS[ufunc], *inputs)

  def __array_function__(self, func, types, args, kwargs):
    if kwargs or len(args) != 1:
      raise NotLowerable('{} with options in a density'.format(func.__name__))
    if func in (np.max, np.amax):
      return Node('max', args[0])
    if func is np.sum:
      return Node('sum', args[0])
    raise NotLowerable('{} in a density'.format(func.__name__))

  def __add__(self, o):
    return Node('add', self, o)

  def __radd__(self, o):
    return Node('add', o, self)

  def __sub__(self, o):
    return Node('sub', self, o)

  def __rsub__(self, o):
    return Node('sub', o, self)


def _same(a, b):
  """Structural equality of traced values."""
  if a is b:
    return True
  if isinstance(a, Node) and isinstance(b, Node):
    return a.op == b.op and len(a.args) == len(b.args) and \
        all(_same(x, y) for x, y in zip(a.args, b.args))
  if isinstance(a, Node) or isinstance(b, Node):
    return False
  return np.array_equal(np.asarray(a), np.asarray(b))


def _lse_operand(out):
  """A from m + log(sum(exp(A - m))) with m = max(A), or logsumexp(A)."""
  if isinstance(out, Node) and out.op == 'lse':
    return out.args[0]
  if not (isinstance(out, Node) and out.op == 'add' and len(out.args) == 2):
    return None
  m, lg = out.args
  if not (isinstance(m, Node) and m.op == 'max'):
    return None
  A = m.args[0]
  ok = isinstance(lg, Node) and lg.op == 'log' and \
      isinstance(lg.args[0], Node) and lg.args[0].op == 'sum'
  ex = lg.args[0].args[0] if ok else None
  ok = ok and isinstance(ex, Node) and ex.op == 'exp'
  df = ex.args[0] if ok else None
  ok = ok and isinstance(df, Node) and df.op == 'sub' and \
      _same(df.args[0], A) and _same(df.args[1], m)
  return A if ok else None


def trace_logsumexp(fn, keys):
  """A log-sum-exp Gaussian mixture written with NumPy (SURVEY App. B H5:
  a = logw + logpdf(x, mu[:, 0], sd) + ...; m + log(sum(exp(a - m))))
  -> gmm target with the SAME summation order, or NotLowerable."""
  import scipy.special

  def logpdf(*args, **kwds):
    x = args[0] if args else kwds.pop('x')
    loc, scale = _loc_scale(args[1:], kwds)
    return Node('logpdf', x, loc, scale)

  def lse(a, *args, **kwds):
    if args or kwds:
      raise NotLowerable('logsumexp with options in a density')
    return Node('lse', a)

  kw = {k: Node('var', k) for k in keys}
  with _patched(scipy.stats.norm, logpdf=logpdf), \
       _patched(scipy.special, logsumexp=lse):
    try:
      out = fn(**kw)
    except NotLowerable:
      raise
    except Exception as e:
      raise NotLowerable('density callable not traceable: {}'.format(e))
  A = _lse_operand(out)
  if A is None:
    raise NotLowerable('density is not a log-sum-exp of component terms')
  terms = []                       # left-associated a = c + t_0 + t_1 + ...
  while isinstance(A, Node) and A.op == 'add':
    terms.append(A.args[1])
    A = A.args[0]
  terms.append(A)
  terms = terms[::-1]
  d = len(keys)
  if len(terms) != d + 1 or isinstance(terms[0], Node):
    raise NotLowerable('mixture must be logw + one logpdf per variable')
  logw = np.asarray(terms[0], np.float64).reshape(-1)
  K = logw.size
  mu = np.empty((K, d))
  sd = None
  for i, t in enumerate(terms[1:]):
    if not (isinstance(t, Node) and t.op == 'logpdf' and
            isinstance(t.args[0], Node) and t.args[0].op == 'var' and
            t.args[0].args[0] == keys[i]):
      raise NotLowerable('mixture terms must be logpdf(x_i, ...) in order')
    _, loc, scale = t.args
    if isinstance(loc, Node) or isinstance(scale, Node):
      raise NotLowerable('mixture loc / scale must be constants')
    mu[:, i] = np.broadcast_to(np.asarray(loc, np.float64), (K,))
    s = np.broadcast_to(np.asarray(scale, np.float64), (K,))
    if sd is not None and not np.array_equal(s, sd):
      raise NotLowerable('mixture sds must be shared across variables')
    sd = np.array(s)
  return {'kind': 'gmm', 'logw': logw, 'mu': mu, 'sd': sd}, 'log'


def is_same_callable(a, b):
  """Bound methods of the same scipy distribution object compare equal."""
  try:
    return a == b
  except Exception:
    return False
