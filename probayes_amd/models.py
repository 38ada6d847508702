"""Descriptor callables: model forms the tracer cannot read from plain code.

Each descriptor is an ordinary Python callable with the reference's calling
convention (keyword arguments named after the variables), so the very same
object can be handed to probayes' set_prob / set_tran and to this package's;
here its `pbh_target` / `pbh_tran` attribute tells the lowering what kernel
form it is.
"""
import numpy as np
import scipy.stats


class GaussianMixtureLogPDF:
  """logsumexp_k(log w_k + sum_i norm.logpdf(x_i, mu_ki, sd_k)): an isotropic
  Gaussian mixture, evaluated as
  m + log(sum(exp(a - m))) with m = max(a)."""

  def __init__(self, keys, weights, means, sds):
    self.keys = list(keys)
    self.logw = np.log(np.asarray(weights, np.float64))
    self.mu = np.asarray(means, np.float64).reshape(len(self.logw),
                                                    len(self.keys))
    self.sd = np.asarray(sds, np.float64).reshape(-1)
    self.pbh_target = {'kind': 'gmm', 'logw': self.logw, 'mu': self.mu,
                       'sd': self.sd}
    self.pbh_pscale = 'log'

  def __call__(self, **kw):
    a = self.logw
    for i, k in enumerate(self.keys):
      a = a + scipy.stats.norm.logpdf(kw[k], self.mu[:, i], self.sd)
    m = np.max(a)
    return m + np.log(np.sum(np.exp(a - m)))


class DiagGaussLogPDF:
  """sum_i norm.logpdf(x_i, mu_i, sigma_i) (Python sum, left to right)."""

  def __init__(self, keys, mu, sigma):
    self.keys = list(keys)
    self.mu = np.asarray(mu, np.float64).reshape(-1)
    self.sigma = np.asarray(sigma, np.float64).reshape(-1)
    self.pbh_target = {'kind': 'diag_gauss', 'mu': self.mu,
                       'sigma': self.sigma}
    self.pbh_pscale = 'log'

  def __call__(self, **kw):
    return sum(scipy.stats.norm.logpdf(kw[k], self.mu[i], self.sigma[i])
               for i, k in enumerate(self.keys))
