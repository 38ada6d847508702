"""RV and RF: the variable / field layer of the SP facade.

RV mirrors probayes rv.py / variable.py for what the MH path reads from it:
the value set and its bound inclusivity (variable.py:352-366: a limit wrapped
in a tuple is exclusive), the (log, exp) change of variable set_ufun
(variable.py:641-697), the transformed length (variable.py:313-342) and the
default uniform prior -log(length) (rv.py:153-166).  RF mirrors rf.py's
set_prob / set_tran / set_delta / set_tfun holders.  `x & y` builds an RF
(ops.py:4-75).
"""
import collections

import numpy as np


class RV:
  """A random variable (rv.py:28)."""

  def __init__(self, name, vtype=float, vset=None, pscale=None, *args, **kwds):
    if vtype in (float, np.float64, 'float'):
      vtype = float
    elif vtype in (int, np.int64, 'int'):
      vtype = int
    else:
      raise NotImplementedError(
          'RV {}: only float and int variables are on the GPU MH path'
          .format(name))
    self.name = str(name)
    self.vtype = vtype
    self.vset = vset
    self.pscale = pscale
    self.ufun = None
    self._log_ufun = False
    if vtype is int:
      self._parse_int_vset(vset)
    else:
      self._parse_vset(vset)

  def _parse_int_vset(self, vset):
    """Non-float value sets (variable.py:169-205, 258-261, 322-329): a
    list / set / range / array of values; vlims = (min, max), length = the
    number of values, both limits inclusive."""
    if vset is None:
      vset = [0, 1]                          # DEFAULT_VSETS[int]
    if isinstance(vset, tuple):
      raise NotImplementedError('RV {}: a tuple vset makes the variable a '
                                'float'.format(self.name))
    vals = sorted(int(v) for v in vset)
    if not vals:
      raise ValueError('RV {}: empty vset'.format(self.name))
    self.vset = vals
    self.vlims = np.array([float(vals[0]), float(vals[-1])])
    self.lo_incl = self.hi_incl = True
    self._int_len = len(vals)

  def _parse_vset(self, vset):
    """Float limits (variable.py:169-205, 262-275): a two-value tuple
    excludes both limits; in a list, a limit wrapped in a tuple is
    exclusive."""
    if vset is None:
      vset = [(-np.inf,), (np.inf,)]         # DEFAULT_VSETS[float]
    if isinstance(vset, tuple):
      if len(vset) != 2:
        raise ValueError('Tuple vsets contain pairs of values, not '
                         '{}'.format(vset))
      vset = [(v,) for v in sorted(vset)]
    if len(vset) != 2:
      raise ValueError('float RV vset needs two limits, got {}'.format(vset))
    lims, incl = [], []
    for v in vset:
      if isinstance(v, tuple):
        lims.append(float(v[0]))
        incl.append(False)
      else:
        lims.append(float(v))
        incl.append(True)
    if lims[1] < lims[0]:                    # variable.py:268-271 re-orders
      lims, incl = lims[::-1], incl[::-1]
    self.vlims = np.array(lims)
    self.lo_incl, self.hi_incl = incl[0], incl[1]

  def set_ufun(self, ufun=None, *args, **kwds):
    """Change of variable (variable.py:641-697).  Only (np.log, np.exp) is
    lowered to the kernels."""
    self.ufun = ufun
    if ufun is None:
      self._log_ufun = False
      return
    if self.vtype is int:
      raise NotImplementedError('RV {}: non-floats do not support '
                                'transformation'.format(self.name))
    fwd, inv = ufun
    if fwd is not np.log or inv is not np.exp:
      raise NotImplementedError(
          'RV {}: only the (np.log, np.exp) ufun is lowered'.format(self.name))
    self._log_ufun = True

  @property
  def log_ufun(self):
    return self._log_ufun

  @property
  def ulims(self):
    """Transformed limits (variable.py:332-335)."""
    return np.log(self.vlims) if self._log_ufun else self.vlims

  @property
  def length(self):
    """max(ulims) - min(ulims) (variable.py:336); the number of values for
    an int variable (variable.py:327)."""
    if self.vtype is int:
      return float(self._int_len)
    ul = self.ulims
    return max(ul) - min(ul)

  @property
  def lhv(self):
    L = self.length
    return np.log(L) if np.isfinite(L) else np.inf

  def __and__(self, other):
    return RF(self, other)

  def __repr__(self):
    return self.name


class RF:
  """A random field of RVs (rf.py:25) holding prob / tran / delta specs."""

  def __init__(self, *args):
    rvs = []
    for a in args:
      if isinstance(a, RV):
        rvs.append(a)
      elif isinstance(a, RF):
        rvs.extend(a.rvs)
      else:
        raise TypeError('RF takes RVs or RFs, not {}'.format(type(a)))
    names = [v.name for v in rvs]
    if len(set(names)) != len(names):
      raise ValueError('repeated variable names {}'.format(names))
    self.rvs = rvs
    self.prob = None
    self.tran = None
    self.tran_kwds = {}
    self.delta = None
    self.delta_args = ()
    self.delta_kwds = {}
    self.tfun = None
    self.Delta = collections.namedtuple('Delta', names)

  @property
  def keylist(self):
    return [v.name for v in self.rvs]

  def __and__(self, other):
    return RF(self, other)

  def set_prob(self, prob=None, *args, **kwds):
    self.prob = (prob, args, kwds)

  def set_tran(self, tran=None, *args, **kwds):
    """rf.py:169-239: a callable, a (forward, reverse) tuple, a scipy
    multivariate_normal (CondCov Gibbs, tsteps=), an RF to delegate to, or a
    covariance matrix: a square array sets its Cholesky factor as the tfun
    (rf.py:210-220) that multiplies every delta (rf.py:340-354)."""
    kwds = dict(kwds)
    self.tran = (tran, args, kwds)
    if isinstance(tran, np.ndarray):
      d = len(self.rvs)
      if tran.ndim != 2 or tran.shape != (d, d):
        raise AssertionError('Non-callable non-scalar tran objects must be a '
                             'square 2D Numpy array of size corresponding to '
                             'number of variables {}'.format(d))
      if kwds.get('tsteps'):
        raise AssertionError('Setting tsteps not supported for covariance '
                             'transitions')
      self.set_tfun(np.linalg.cholesky(tran))

  def set_delta(self, delta=None, *args, **kwds):
    """field.py:220-317: scalar in a tuple (spherical), in a list (uniform
    per variable), or a callable returning Delta(...)."""
    self.delta = delta
    self.delta_args = args
    self.delta_kwds = dict(kwds)

  def set_tfun(self, tfun=None, *args, **kwds):
    """rf.py:247-304.  A non-callable tfun is a triangular (LU) factor."""
    if isinstance(tfun, np.ndarray):
      d = len(self.rvs)
      if tfun.ndim != 2 or tfun.shape != (d, d) or not (
          np.allclose(tfun, np.tril(tfun)) or np.allclose(tfun, np.triu(tfun))):
        raise AssertionError('Non-callable tran objects must be a triangular '
                             '2D Numpy array of size corresponding to number '
                             'of variables {}'.format(d))
      tfun = np.array(tfun, dtype=np.float64)
    self.tfun = None if tfun is None else (tfun, args, kwds)

  @property
  def lud(self):
    """The triangular tfun factor, or None (rf.py:347-349)."""
    if self.tfun is not None and isinstance(self.tfun[0], np.ndarray):
      return self.tfun[0]
    return None

  def __repr__(self):
    return '&'.join(self.keylist)
