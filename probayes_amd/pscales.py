"""pscale conventions (host side), restating probayes pscales.py:21-131.

A float pscale is a linear coefficient, a complex one a log offset; 'log' /
'ln' / 0 mean natural log probabilities (eval_pscale, pscales.py:21-41).  Only
the conversions the facade needs on results are here; the per-step
arithmetic of the acceptance lives in the HIP kernels.
"""
import numpy as np

NEARLY_POSITIVE_ZERO = 2.2250738585072014e-308
NEARLY_POSITIVE_INF = 1.7976931348623158e+308
NEARLY_NEGATIVE_INF = -NEARLY_POSITIVE_INF
LOG_NEARLY_POSITIVE_INF = np.log(NEARLY_POSITIVE_INF)


def is_log(pscale):
  """True for a log pscale ('log', 'ln', 0, 0j or any complex)."""
  if pscale is None:
    return False
  if isinstance(pscale, str):
    if pscale in ('log', 'ln'):
      return True
    if pscale == 'lin':
      return False
    raise ValueError('Cannot evaluate pscale={}'.format(pscale))
  if isinstance(pscale, complex):
    return True
  if pscale == 0:
    return True
  return False


def pscale_name(pscale):
  return 'log' if is_log(pscale) else 'lin'


def exp_logp(logp):
  """pscales.py:56-65."""
  logp = np.asarray(logp, dtype=np.float64)
  out = np.full(logp.shape, NEARLY_POSITIVE_INF)
  ok = logp <= LOG_NEARLY_POSITIVE_INF
  out[ok] = np.exp(logp[ok])
  return out if out.ndim else float(out)


def log_prob(prob):
  """pscales.py:44-53."""
  prob = np.asarray(prob, dtype=np.float64)
  out = np.full(prob.shape, NEARLY_NEGATIVE_INF)
  ok = prob >= NEARLY_POSITIVE_ZERO
  out[ok] = np.log(prob[ok])
  return out if out.ndim else float(out)


def rescale(prob, pscale, rtype=None):
  """rescale(prob, pscale, rtype) between the log and unit linear scales
  (pscales.py:100-131 with unit coefficients)."""
  p_log, r_log = is_log(pscale), is_log(rtype)
  if p_log == r_log:
    return prob
  return exp_logp(prob) if p_log else log_prob(prob)
