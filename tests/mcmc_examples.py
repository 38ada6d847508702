"""The examples/mcmc workloads as builder functions of the API module `pb`.

Each builder restates one reference script (cited per builder) with only the
step counts and seeds changed.  `pb` is either the reference package (run by
tools/gen_golden.py in the build container to record tests/golden/) or
probayes_amd (run by the facade tests) -- the same code drives both, so the
facade tests read like the reference's own example scripts.
"""
import numpy as np
import scipy
import scipy.stats
import scipy.special


# ----------------------------------------------------------------------------
# Model builders.  Each returns (process, init, extra, sampler_kwds, keys)
# ----------------------------------------------------------------------------
def metrohast_norm1d(pb, params):
  """examples/mcmc/metrohast_norm1d.py:13-40 (cfg1)."""
  x_obs = params['x_obs']
  mu = pb.RV('mu', vtype=float, vset=(40, 60), pscale='log')
  sigma = pb.RV('sigma', vtype=float, vset=(5, 20.), pscale='log')
  x = pb.RV('x', vtype=float, vset=(-np.inf, np.inf))
  sigma.set_ufun((np.log, np.exp))
  paras = pb.RF(mu, sigma)
  stats = pb.RF(x)
  process = pb.SP(stats, paras)
  process.set_prob(scipy.stats.norm.logpdf,
                   order={'x': 0, 'mu': 'loc', 'sigma': 'scale'})
  tran = lambda **x: 1.
  paras.set_tran((tran, tran))
  paras.set_delta((0.005,), scale=True)
  process.set_tran(paras)
  process.set_delta(paras)
  process.set_scores('hastings')
  process.set_update('metropolis')
  init = {mu: 50., sigma: 12.5}
  return process, init, {x: x_obs}, {'iid': True, 'joint': True}, ['mu', 'sigma']


def mcmc_prob2(pb, params):
  """examples/mcmc/mcmc_prob2.py:19-31."""
  def q(**kwds):
    x, xprime = kwds['x'], kwds["x'"]
    return scipy.stats.norm.pdf(xprime, loc=x, scale=1.)
  x = pb.RV('x', vtype=float, vset=(-np.inf, np.inf))
  process = pb.SP(x)
  process.set_prob(scipy.stats.norm.pdf, loc=2, scale=np.sqrt(2),
                   order={'x': 0})
  process.set_tran(q)
  lambda_delta = lambda: process.Delta(x=scipy.stats.norm.rvs(loc=0., scale=1.))
  process.set_delta(lambda_delta)
  process.set_scores('hastings')
  process.set_update('metropolis')
  return process, {'x': 0.}, None, {}, ['x']


def mcmc_prob3(pb, params):
  """examples/mcmc/mcmc_prob3.py:27-39 (uniform target, linear pscale)."""
  def q(**kwds):
    x, xprime = kwds['x'], kwds["x'"]
    return scipy.stats.norm.pdf(xprime, loc=x, scale=1.)
  x = pb.RV('x', vtype=float, vset=(-np.inf, np.inf))
  process = pb.SP(x)
  process.set_prob(scipy.stats.uniform.pdf, loc=3., scale=4.,
                   order={'x': 0})
  process.set_tran(q)
  lambda_delta = lambda: process.Delta(x=scipy.stats.norm.rvs(loc=0., scale=1.))
  process.set_delta(lambda_delta)
  process.set_scores('hastings')
  process.set_update('metropolis')
  return process, {'x': 5.}, None, {}, ['x']


def _q2(prop_stdv, xoff=0.):
  def q(**kwds):
    x, xprime = kwds['x'], kwds["x'"]
    y, yprime = kwds['y'], kwds["y'"]
    return scipy.stats.norm.pdf(yprime, loc=y, scale=prop_stdv) * \
           scipy.stats.norm.pdf(xprime, loc=x+xoff, scale=prop_stdv)
  return q


def mcmc_prob4a(pb, params):
  """examples/mcmc/mcmc_prob4a.py:33-48 (2-D mvn target, permuted density)."""
  prop_stdv = np.sqrt(1)
  x = pb.RV('x', vtype=float, vset=(-np.inf, np.inf))
  y = pb.RV('y', vtype=float, vset=(-np.inf, np.inf))
  process = pb.SP(x & y)
  process.set_prob(scipy.stats.multivariate_normal, [0., 0.],
                   [[2.0, 1.2], [1.2, 2.0]])
  process.set_tran(_q2(prop_stdv))
  lambda_delta = lambda: process.Delta(
      x=scipy.stats.norm.rvs(loc=0., scale=prop_stdv),
      y=scipy.stats.norm.rvs(loc=0., scale=prop_stdv))
  process.set_delta(lambda_delta)
  process.set_scores('hastings')
  process.set_update('metropolis')
  return process, {'x': 0., 'y': 1.}, None, {}, ['x', 'y']


def mcmc_prob4b(pb, params):
  """examples/mcmc/mcmc_prob4b.py:31-51 (top-hat product target)."""
  prop_stdv = np.sqrt(1)
  def p(**kwds):
    return scipy.stats.uniform.pdf(kwds['x'], loc=3., scale=4.) * \
           scipy.stats.uniform.pdf(kwds['y'], loc=1., scale=8.)
  x = pb.RV('x', vtype=float, vset=(-np.inf, np.inf))
  y = pb.RV('y', vtype=float, vset=(-np.inf, np.inf))
  process = pb.SP(x & y)
  process.set_prob(p)
  process.set_tran(_q2(prop_stdv))
  lambda_delta = lambda: process.Delta(
      x=scipy.stats.norm.rvs(loc=0., scale=prop_stdv),
      y=scipy.stats.norm.rvs(loc=0., scale=prop_stdv))
  process.set_delta(lambda_delta)
  process.set_scores('hastings')
  process.set_update('metropolis')
  return process, {'x': 5., 'y': 5.}, None, {}, ['x', 'y']


def mcmc_prob6(pb, params):
  """examples/mcmc/mcmc_prob6.py:44-61 (asymmetric (q, r) tuple tran)."""
  prop_stdv = np.sqrt(1)
  x = pb.RV('x', vtype=float, vset=(-np.inf, np.inf))
  y = pb.RV('y', vtype=float, vset=(-np.inf, np.inf))
  process = pb.SP(x & y)
  process.set_prob(scipy.stats.multivariate_normal, [0., 0.],
                   [[2.0, 1.2], [1.2, 2.0]])
  process.set_tran((_q2(prop_stdv, 2.), _q2(prop_stdv, -2.)))
  lambda_delta = lambda: process.Delta(
      x=scipy.stats.norm.rvs(loc=-2, scale=prop_stdv),
      y=scipy.stats.norm.rvs(loc=0., scale=prop_stdv))
  process.set_delta(lambda_delta)
  process.set_scores('hastings')
  process.set_update('metropolis')
  return process, {'x': 0., 'y': 1.}, None, {}, ['x', 'y']


def gibbs_norm2d(pb, params):
  """examples/mcmc/gibbs_norm2d.py:9-21."""
  lims = (-10., 10.)
  means = [0.5, -0.5]
  covar = [[1.5, -1.0], [-1.0, 2.]]
  x = pb.RV('x', vtype=float, vset=lims)
  y = pb.RV('y', vtype=float, vset=lims)
  process = pb.SP(x & y)
  process.set_prob(scipy.stats.multivariate_normal, means, covar)
  process.set_tran(scipy.stats.multivariate_normal, means, covar, tsteps=1)
  process.set_scores('gibbs')
  return process, {'x': 0., 'y': 1.}, None, {}, ['x', 'y']


def diag10(pb, params):
  """10-dim diagonal Gaussian, callable N(0, 0.5^2) delta."""
  mus, sigmas = params['mu'], params['sigma']
  keys = ['x{}'.format(i) for i in range(len(mus))]
  xs = [pb.RV(k, vtype=float, vset=(-np.inf, np.inf)) for k in keys]
  process = pb.SP(pb.RF(*xs))
  def lp(**kw):
    return sum(scipy.stats.norm.logpdf(kw[k], mus[i], sigmas[i])
               for i, k in enumerate(keys))
  process.set_prob(lp, pscale='log')
  process.set_tran(lambda **kw: 1.)
  process.set_delta(lambda: process.Delta(
      **{k: scipy.stats.norm.rvs(scale=params['step']) for k in keys}))
  process.set_scores('hastings')
  process.set_update('metropolis')
  return process, {k: 0. for k in keys}, None, {}, keys


def gibbs8(pb, params):
  """8-dim mvn CondCov Gibbs."""
  mean, cov = params['mean'], params['cov']
  keys = ['x{}'.format(i) for i in range(len(mean))]
  xs = [pb.RV(k, vtype=float, vset=(-20., 20.)) for k in keys]
  process = pb.SP(pb.RF(*xs))
  process.set_prob(scipy.stats.multivariate_normal, mean, cov)
  process.set_tran(scipy.stats.multivariate_normal, mean, cov, tsteps=1)
  process.set_scores('gibbs')
  return process, {k: 0. for k in keys}, None, {}, keys


def gmm2(pb, params):
  """3-component 2-D isotropic Gaussian mixture."""
  logw, mu, sd = np.log(params['w']), params['mu'], params['sd']
  x = pb.RV('x', vtype=float, vset=(-np.inf, np.inf))
  y = pb.RV('y', vtype=float, vset=(-np.inf, np.inf))
  process = pb.SP(x & y)
  def logp(**kw):
    a = logw + scipy.stats.norm.logpdf(kw['x'], mu[:, 0], sd) + \
               scipy.stats.norm.logpdf(kw['y'], mu[:, 1], sd)
    m = np.max(a)
    return m + np.log(np.sum(np.exp(a - m)))
  process.set_prob(logp, pscale='log')
  process.set_tran(lambda **kw: 1.)
  step = params['step']
  process.set_delta(lambda: process.Delta(
      x=scipy.stats.norm.rvs(scale=step), y=scipy.stats.norm.rvs(scale=step)))
  process.set_scores('hastings')
  process.set_update('metropolis')
  return process, {'x': 0., 'y': 0.}, None, {}, ['x', 'y']


def _cfg3_params():
  rs = np.random.RandomState(123)
  A = rs.normal(size=(8, 8))
  cov = A.dot(A.T) / 8 + 0.5 * np.eye(8)
  mean = 0.5 * rs.normal(size=8)
  return {'mean': mean, 'cov': cov}


WORKLOADS = {
  # name: (builder, params, n_chains, n_steps, seed0)
  'metrohast_norm1d': (metrohast_norm1d,
                       {'x_obs': np.random.RandomState(1).normal(50., 10., 60)},
                       32, 256, 1000),
  'mcmc_prob2': (mcmc_prob2, {}, 32, 256, 2000),
  'mcmc_prob3': (mcmc_prob3, {}, 16, 256, 3000),
  'mcmc_prob4a': (mcmc_prob4a, {}, 16, 256, 4000),
  'mcmc_prob4b': (mcmc_prob4b, {}, 16, 256, 4500),
  'mcmc_prob6': (mcmc_prob6, {}, 16, 256, 6000),
  'gibbs_norm2d': (gibbs_norm2d, {}, 16, 256, 7000),
  'diag10': (diag10, {'mu': np.linspace(-1., 1., 10),
                      'sigma': np.linspace(0.5, 2., 10), 'step': 0.5},
             32, 256, 8000),
  'gibbs8': (gibbs8, _cfg3_params(), 16, 256, 9000),
  'gmm2': (gmm2, {'w': np.array([0.3, 0.5, 0.2]),
                  'mu': np.array([[-2., 0.], [2., 1.], [0., -2.5]]),
                  'sd': np.array([0.6, 0.8, 0.5]), 'step': 0.7},
           32, 256, 10000),
}


def gibbs_sweep2(pb, params):
  """examples/cov/multinorm_rw.py:6-15 model (CondCov tran without tsteps:
  every coordinate per step, rf.py:446-452) driven through SP with gibbs
  scores."""
  lims = (-10., 10.)
  means = [0.5, -0.5]
  covar = [[1.5, -1.0], [-1.0, 2.]]
  x = pb.RV('x', vtype=float, vset=lims)
  y = pb.RV('y', vtype=float, vset=lims)
  process = pb.SP(x & y)
  process.set_prob(scipy.stats.multivariate_normal, means, covar)
  process.set_tran(scipy.stats.multivariate_normal, means, covar)
  process.set_scores('gibbs')
  return process, {'x': 0., 'y': 0.}, None, {}, ['x', 'y']


WORKLOADS['gibbs_sweep2'] = (gibbs_sweep2, {}, 16, 256, 11000)


# ----------------------------------------------------------------------------
# Covariance-matrix random walk: RF.set_tran(ndarray)
# sets the Cholesky factor as the RF's tfun (rf.py:210-220) and RF.eval_delta
# multiplies every base delta by it (rf.py:340-354); the SP reaches the RF's
# tran and delta through its subfield name (sd.py:97-105, dependence.py:316-
# 339), which is the route that runs (SP.set_tran(ndarray) itself fails in
# leafs_roots on the array comparison).
# ----------------------------------------------------------------------------
def covrw2(pb, params):
  """examples/cov/multinorm_rw.py:6-15 model (mvn target at the permuted
  vector, App. A-4) with a covariance RW proposal: callable N(0, 0.5^2)
  Delta times chol(cov)."""
  lims = (-10., 10.)
  means = [0.5, -0.5]
  covar = np.array([[1.5, -1.0], [-1.0, 2.]])
  x = pb.RV('x', vtype=float, vset=lims)
  y = pb.RV('y', vtype=float, vset=lims)
  xy = x & y
  xy.set_tran(covar)
  step = params['step']
  xy.set_delta(lambda: xy.Delta(x=scipy.stats.norm.rvs(scale=step),
                                y=scipy.stats.norm.rvs(scale=step)))
  process = pb.SP(xy)
  process.set_prob(scipy.stats.multivariate_normal, means, covar)
  process.set_tran('leafs')
  process.set_delta('leafs')
  process.set_scores('hastings')
  process.set_update('metropolis')
  return process, {'x': 0., 'y': 0.}, None, {}, ['x', 'y']


def covrw5(pb, params):
  """5-dim diagonal-Gaussian target (the H3 form at d = 5) under a
  covariance RW proposal from a spherical tuple delta (field.py:509-531)
  times chol(cov) (rf.py:340-354)."""
  mus, sigmas, cov = params['mu'], params['sigma'], params['cov']
  keys = ['x{}'.format(i) for i in range(len(mus))]
  xs = [pb.RV(k, vtype=float, vset=(-10., 10.)) for k in keys]
  rf = pb.RF(*xs)
  rf.set_tran(cov)
  rf.set_delta((params['step'],))
  process = pb.SP(rf)
  def lp(**kw):
    return sum(scipy.stats.norm.logpdf(kw[k], mus[i], sigmas[i])
               for i, k in enumerate(keys))
  process.set_prob(lp, pscale='log')
  process.set_tran('leafs')
  process.set_delta('leafs')
  process.set_scores('hastings')
  process.set_update('metropolis')
  return process, {k: 0. for k in keys}, None, {}, keys


def _covrw5_params():
  rs = np.random.RandomState(55)
  A = rs.normal(size=(5, 5))
  return {'mu': np.linspace(-1., 1., 5), 'sigma': np.linspace(0.5, 2., 5),
          'cov': A.dot(A.T) / 5 + 0.25 * np.eye(5), 'step': 0.6}


WORKLOADS['covrw2'] = (covrw2, {'step': 0.5}, 16, 256, 12000)
WORKLOADS['covrw5'] = (covrw5, _covrw5_params(), 16, 256, 13000)


def _linreg_params():
  rs = np.random.RandomState(321)
  x_obs = rs.normal(0, 1, size=60)
  y_obs = rs.normal(1.5 * x_obs - 1., 0.5)
  return {'x_obs': x_obs, 'y_obs': y_obs,
          'init': np.array([-0.9, 1.4, 0.6])}


def linreg_cond(x_obs, y_obs):
  """The conditional sampler of examples/mcmc/gibbs_linreg.py:34-62 (cond_reg)
  with the example's default hyper-parameters, closed over the data size."""
  rand_size = len(x_obs)

  def cond_reg(x, y, beta_0, beta_1, y_sigma, unknown,
               beta_0_mu=0, beta_0_sigma=1, beta_1_mu=0, beta_1_sigma=1.,
               y_sigma_alpha=1., y_sigma_beta=1.):
    if unknown == 'y_sigma':
      cond_alpha = y_sigma_alpha + 0.5 * rand_size
      cond_beta = y_sigma_beta + 0.5 * np.sum((y - beta_0 - beta_1 * x) ** 2)
      return 1 / np.sqrt(np.random.gamma(cond_alpha, 1 / cond_beta))
    y_prec = 1 / (y_sigma ** 2)
    if unknown == 'beta_0':
      beta_0_prec = 1 / (beta_0_sigma ** 2)
      cond_var = 1 / (beta_0_prec + rand_size * y_prec)
      cond_mu = (beta_0_prec * beta_0_mu + y_prec * np.sum(y - beta_1 * x)) \
          * cond_var
      return np.random.normal(cond_mu, np.sqrt(cond_var))
    if unknown == 'beta_1':
      beta_1_prec = 1 / (beta_1_sigma ** 2)
      cond_var = 1 / (beta_1_prec + y_prec * np.sum(x ** 2))
      cond_mu = (beta_1_prec * beta_1_mu + y_prec * np.sum(x * (y - beta_0))) \
          * cond_var
      return np.random.normal(cond_mu, np.sqrt(cond_var))
    raise ValueError("Unknown unknown: {}".format(unknown))
  return cond_reg


def gibbs_linreg(pb, params):
  """examples/mcmc/gibbs_linreg.py:26-80 (user-tfun Gibbs, rf.py:464-487),
  data from a fixed RandomState instead of the global stream."""
  x_obs, y_obs = params['x_obs'], params['y_obs']
  x = pb.RV('x', vtype=float, vset=[-3, 3])
  y = pb.RV('y', vtype=float, vset=[-np.inf, np.inf])
  beta_0 = pb.RV('beta_0', vtype=float, vset=[-6., 6.])
  beta_1 = pb.RV('beta_1', vtype=float, vset=[-6., 6.])
  y_sigma = pb.RV('y_sigma', vtype=float, vset=[(0.001), 10.])

  def norm_reg(x, y, beta_0, beta_1, y_sigma):
    return scipy.stats.norm.logpdf(y, loc=beta_0 + beta_1 * x, scale=y_sigma)

  stats = x & y
  paras = beta_0 & beta_1 & y_sigma
  cond = params['cond'](len(x_obs)) if 'cond' in params else \
      linreg_cond(x_obs, y_obs)
  paras.set_tfun(cond, tsteps=1, x=x_obs, y=y_obs)
  process = pb.SP(stats, paras)
  process.set_tfun(paras)
  process.set_prob(norm_reg, pscale='log')
  process.set_scores('gibbs')
  init = dict(zip(['beta_0', 'beta_1', 'y_sigma'], params['init']))
  return (process, init, {'x,y': [x_obs, y_obs]},
          {'iid': True, 'joint': True}, ['beta_0', 'beta_1', 'y_sigma'])


# user-tfun Gibbs: lowered by probayes_amd.linreg, not the generic spec
# (oracle/linreg.py, tests/test_linreg.py)
TFUN_WORKLOADS = {'gibbs_linreg': (gibbs_linreg, _linreg_params(), 8, 96, 14000)}


# ----------------------------------------------------------------------------
# Delta forms beyond the callable / plain tuple / plain list:
# bound=True (variable.py:700-739: clamp closed limits, bounce exclusive
# ones), per-variable dict deltas (field.py:266-274, variable.py:600-640:
# tuple = random polarity, list = uniform or, for int variables, randint,
# bare scalar = fixed step), the unscaled-override dict args[0]
# (field.py:276-306) and bare scalar Field deltas.  The models restate
# examples/omc/omc_rw_circle.py:16-22 (tuple vsets, spherical delta,
# bound=True) and examples/markov/markov_delta.py:32 (list delta, scale and
# bound) on small diagonal-Gaussian densities so that chains reach the limits.
# ----------------------------------------------------------------------------
def _diag_lp(keys, mus, sigmas):
  def lp(**kw):
    return sum(scipy.stats.norm.logpdf(kw[k], mus[i], sigmas[i])
               for i, k in enumerate(keys))
  return lp


def _delta_model(pb, rvs, mus, sigmas, init):
  keys = [v.name for v in rvs]
  process = pb.SP(pb.RF(*rvs))
  process.set_prob(_diag_lp(keys, mus, sigmas), pscale='log')
  process.set_tran(lambda **kw: 1.)
  process.set_scores('hastings')
  process.set_update('metropolis')
  return process, dict(zip(keys, init)), None, {}, keys


def bound_sphere2(pb, params):
  """omc_rw_circle.py:16-22: tuple vsets (both limits exclusive) and
  set_delta((0.15 r,), bound=True) -> proposals leaving the box bounce back."""
  x = pb.RV('x', vtype=float, vset=(-1., 1.))
  y = pb.RV('y', vtype=float, vset=(-1., 1.))
  out = _delta_model(pb, [x, y], [0.7, -0.6], [0.4, 0.5], [0., 0.])
  out[0].set_delta((params['step'],), bound=True)
  return out


def _three_vsets(pb):
  return [pb.RV('x', vtype=float, vset=[(-1.,), 1.]),    # lower exclusive
          pb.RV('y', vtype=float, vset=[-1., (1.,)]),    # upper exclusive
          pb.RV('z', vtype=float, vset=[0., 2.])]        # closed


def bound_list3(pb, params):
  """markov_delta.py:32 form on a field: set_delta([d], {'z': [dz]},
  scale=True, bound=True): uniform deltas scaled by length except the
  unscaled override, one-sided bounces and a clamp."""
  out = _delta_model(pb, _three_vsets(pb), [-0.8, 0.8, 1.9], [0.5, 0.5, 0.6],
                     [0., 0., 1.])
  out[0].set_delta([0.2], {'z': 0.15}, scale=True, bound=True)
  return out


def pervar3(pb, params):
  """Per-variable deltas as a Delta instance (field.py:266-274): x random
  polarity, y uniform, z a fixed step scaled by its length, all bounded."""
  out = _delta_model(pb, _three_vsets(pb), [-0.8, 0.8, 1.9], [0.5, 0.5, 0.6],
                     [0., 0., 1.])
  p = out[0]
  p.set_delta(p.Delta(x=(0.25,), y=[0.3], z=0.05), scale=True, bound=True)
  return out


def dict3(pb, params):
  """A dict delta: field.py:262-263 converts it to a Delta but tests the
  ORIGINAL argument, so it takes the tuple (spherise) branch with no
  per-variable deltas set; eval_delta then yields Delta(None, ...) and
  apply_delta leaves every value unchanged (variable.py:660-672)."""
  out = _delta_model(pb, _three_vsets(pb), [-0.8, 0.8, 1.9], [0.5, 0.5, 0.6],
                     [0.1, 0.2, 1.])
  out[0].set_delta({'x': (0.25,), 'y': [0.3], 'z': 0.05}, bound=True)
  return out


def fixed2(pb, params):
  """Bare scalar Field delta (fixed step) with an unscaled override."""
  x = pb.RV('x', vtype=float, vset=[-1., 1.])
  y = pb.RV('y', vtype=float, vset=[-1., 1.])
  out = _delta_model(pb, [x, y], [0.3, -0.2], [0.5, 0.4], [0., 0.])
  out[0].set_delta(0.02, {'y': -0.03}, scale=True, bound=True)
  return out


def randint2(pb, params):
  """An int variable's list delta draws np.random.randint(-d, d)
  (variable.py:630-631); a zero draw is redrawn once by apply_delta's
  `delta or self._delta` (variable.py:660-667); bound clamps the int to its
  value-set limits."""
  n = pb.RV('n', vtype=int, vset=range(0, 21))
  x = pb.RV('x', vtype=float, vset=(-np.inf, np.inf))
  out = _delta_model(pb, [n, x], [12., 0.], [3., 1.], [0, 0.])
  p = out[0]
  p.set_delta(p.Delta(n=[3], x=[0.5]), bound=True)
  return out


DELTA_WORKLOADS = {
  'bound_sphere2': (bound_sphere2, {'step': 0.15}, 16, 256, 15000),
  'bound_list3': (bound_list3, {}, 16, 256, 16000),
  'pervar3': (pervar3, {}, 16, 256, 17000),
  'fixed2': (fixed2, {}, 8, 128, 18000),
  'dict3': (dict3, {}, 8, 64, 18500),
  'randint2': (randint2, {}, 16, 256, 19000),
}

# Consecutive samplers on ONE process share the RF's CondCov cycle phase
# (rf.py:446-452 __cond_mod) and NumPy's global stream: name -> (base
# workload, segment lengths, chains)
SEGMENTED = {
  'gibbs_norm2d_seg': ('gibbs_norm2d', (7, 10), 6),
  'gibbs_linreg_seg': ('gibbs_linreg', (4, 5, 7), 4),
}
