"""Restatement of the reference's covariance-conditioned Gibbs step.

CondCov.__init__ (cond_cov.py:22-39) precomputes per coordinate i the regression
row coef_i = Sigma_{i,-i} Sigma_{-i,-i}^{-1}, the Schur standard deviation and
the cdf limits of the recentred bounds.  Each SP step (rf.py:446-458 cycling one
coordinate per step, per-RF counter) draws u ~ U(cdf_lo, cdf_hi) and sets
x_i = norm.ppf(u, mu_i + coef_i.(x_-i - mu_-i), sd_i) (cond_cov.py:42-65).
Scores/threshold/update are nan/nan/True (sp_utils.py:75-84).  v.prob is the
mvn pdf at the permuted vector (prob.py:349-358, App. A-4).
TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).
"""
import numpy as np
import scipy.stats

from oracle.mh import mvn_perm


def condcov_tables(mean, cov, lo, hi):
  """cond_cov.py:22-39 verbatim in NumPy: (coef[d, d-1], stdv[d], cdfs[d, 2])."""
  mean = np.atleast_1d(np.asarray(mean, np.float64))
  cov = np.atleast_2d(np.asarray(cov, np.float64))
  lims = np.stack([np.asarray(lo, np.float64), np.asarray(hi, np.float64)], -1)
  lims = np.atleast_2d(lims) - np.expand_dims(mean, -1)
  n = len(mean)
  stdv = np.empty(n, dtype=float)
  coef = []
  for i in range(n):
    ll = np.delete(cov[:, i].reshape([n, 1]), (i), axis=0)
    ru = np.delete(cov[i, :].reshape([1, n]), (i), axis=1)
    c = np.delete(np.delete(cov, (i), axis=1), (i), axis=0)
    coef.append(ru.dot(np.linalg.inv(c)))
    stdv[i] = np.sqrt(cov[i, i] - coef[i].dot(ll).item())
  cdfs = np.array([scipy.stats.norm.cdf(lim, loc=0., scale=stdv[i])
                   for i, lim in enumerate(lims)])
  return coef, stdv, cdfs


def run_gibbs(spec, init, streams, step0=0):
  """T coordinate steps for N chains; streams [T, tsteps, N] of raw uniforms.
  step0: SP steps the RF already made, i.e. the cycle phase __cond_mod of
  rf.py:446-452 at which this sampler starts (it persists on the RF across
  samplers)."""
  prop = spec['proposal']
  d = int(spec['dim'])
  T, _, N = streams.shape
  mean = np.asarray(prop['mean'], np.float64)
  coef, stdv, cdfs = condcov_tables(mean, prop['cov'], prop['lo'], prop['hi'])
  tsteps = int(prop.get('tsteps', 1))
  x = np.array(np.asarray(init, np.float64).reshape(N, d))
  mvn = scipy.stats.multivariate_normal(np.asarray(spec['target']['mean']),
                                        np.asarray(spec['target']['cov']))
  perm = mvn_perm(d)
  out = {'v_x': np.empty((N, T, d)), 'v_p': np.empty((N, T)),
         'u': np.ones((N, T), np.uint8)}
  nblk = -(-d // tsteps)
  for c in range(N):
    cond_mod = (int(step0) % nblk) * tsteps
    xc = x[c]
    for t in range(T):
      for j, key in enumerate(range(cond_mod, min(cond_mod + tsteps, d))):
        dmu = np.empty((d, 1), dtype=float)
        for i in range(d):
          if i != key:
            dmu[i] = xc[i] - mean[i]
        dmu = np.delete(dmu, (key), axis=0)
        lims = cdfs[key]
        u = streams[t, j, c]
        cdf = lims[0] + (lims[1] - lims[0]) * u     # legacy uniform(lo, hi)
        m = mean[key] + coef[key].dot(dmu).item()   # float(1x1 array)
        xc[key] = scipy.stats.norm.ppf(cdf, loc=m, scale=stdv[key])
      cond_mod += tsteps
      if cond_mod >= d:
        cond_mod = 0
      out['v_x'][c, t] = xc
      out['v_p'][c, t] = mvn.pdf(xc[perm].reshape((1,) * d + (d,)))
  out['p_x'], out['p_p'] = out['v_x'], out['v_p']
  return out
