"""Restatement of the reference's user-tfun Gibbs path for the conjugate
linear regression of examples/mcmc/gibbs_linreg.py.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Path: SP.next -> RF.eval_tfun (rf.py:413-462): the paras RF (beta_0 & beta_1 &
y_sigma) calls the user conditional `cond_reg(succ_vals, unknown=key, x=, y=)`
for ONE key per step (tsteps=1; keys cycle beta_0, beta_1, y_sigma through the
RF's __cond_mod, rf.py:446-452).  The conditional draws (gibbs_linreg.py:34-62):
  y_sigma: 1 / sqrt(np.random.gamma(a + n/2, 1 / (b + 0.5 sum((y-b0-b1 x)^2))))
  beta_0 : np.random.normal((m0 p0 + yp sum(y - b1 x)) v, sqrt(v)),
           v = 1 / (p0 + n yp), yp = 1 / y_sigma^2, p0 = 1 / s0^2
  beta_1 : np.random.normal((m1 p1 + yp sum(x (y - b0))) v, sqrt(v)),
           v = 1 / (p1 + yp sum(x^2))
Gibbs scores / thresh / update are None / None / True (sp_utils.py:75-84), so
every step is accepted.  v.prob is the iid log-likelihood sum over the
observations (RF._eval_iid, rf.py:541-562; PD.prod pd.py:368) of
norm.logpdf(y, b0 + b1 x, y_sigma), then joint=True adds the uniform log prior
-log(hi - lo) of each parameter root in RF order (rv_utils.py:30-38).

Random draws are NumPy's legacy ones: normal(loc, scale) = loc + scale * gauss,
gamma(shape, scale) = scale * standard_gamma(shape) (numpy 2.2.6
legacy-distributions.c).  Because the gamma shape a + n/2 does not depend on
the state, the per-step standard draws form a state-independent replay stream
[T][N]: gauss for beta steps, standard_gamma(a + n/2) for y_sigma steps.
"""
import numpy as np
import scipy.stats

KEYS = ('beta_0', 'beta_1', 'y_sigma')
# cond_reg defaults (gibbs_linreg.py:34-36) and the RV vsets (:27-30).
HYPER = {'beta_0_mu': 0., 'beta_0_sigma': 1., 'beta_1_mu': 0.,
         'beta_1_sigma': 1., 'y_sigma_alpha': 1., 'y_sigma_beta': 1.}
VSETS = ((-6., 6.), (-6., 6.), (0.001, 10.))


def linreg_streams(seeds, n_steps, n_obs, hyper=HYPER, cond_mod=0):
  """Per-chain RandomState(seed) standard draws in the reference's order."""
  alpha = hyper['y_sigma_alpha'] + 0.5 * n_obs
  out = np.empty((n_steps, len(seeds)), np.float64)
  for c, s in enumerate(seeds):
    rs = np.random.RandomState(int(s))
    for t in range(n_steps):
      if (t + cond_mod) % 3 == 2:
        out[t, c] = rs.standard_gamma(alpha)
      else:
        out[t, c] = rs.standard_normal()
  return out


NEARLY_NEGATIVE_INF = -1.7976931348623158e+308     # constants.py:31


def log_prior(vsets=VSETS):
  """joint=True uniform root priors, added one by one (rv_utils.py:30-38)."""
  return [-np.log(hi - lo) for lo, hi in vsets]


def prior_terms(vals, vsets=VSETS):
  """uniform_prob (rv_utils.py:30-38) per parameter: -log L inside the closed
  vset, NEARLY_NEGATIVE_INF outside."""
  return [np.where((v >= lo) & (v <= hi), q, NEARLY_NEGATIVE_INF)
          for v, (lo, hi), q in zip(vals, vsets, log_prior(vsets))]


def loglik(x_obs, y_obs, b0, b1, ys):
  """rf.py:541-562 iid sum of norm.logpdf(y, b0 + b1 x, ys) per chain."""
  loc = b0[:, None] + b1[:, None] * x_obs[None, :]
  return np.sum(scipy.stats.norm.logpdf(y_obs[None, :], loc=loc,
                                        scale=ys[:, None]), axis=1)


def run_linreg(x_obs, y_obs, init, streams, hyper=HYPER, vsets=VSETS,
               cond_mod=0):
  """Vectorised over chains.  init [N, 3]; streams [T, N].
  Returns v_x [N, T, 3] and v_p [N, T] like the golden traces."""
  x_obs = np.asarray(x_obs, np.float64)
  y_obs = np.asarray(y_obs, np.float64)
  n = len(x_obs)
  b0, b1, ys = (np.array(init[:, k], np.float64) for k in range(3))
  h = hyper
  sxx = np.sum(x_obs ** 2)
  T, N = streams.shape
  vx = np.empty((N, T, 3))
  vp = np.empty((N, T))
  for t in range(T):
    z = streams[t]
    key = (t + cond_mod) % 3
    if key == 2:
      alpha = h['y_sigma_alpha'] + 0.5 * n
      r = y_obs[None, :] - b0[:, None] - b1[:, None] * x_obs[None, :]
      beta = h['y_sigma_beta'] + 0.5 * np.sum(r ** 2, axis=1)
      del alpha
      ys = 1 / np.sqrt((1 / beta) * z)
    else:
      yp = 1 / (ys ** 2)
      if key == 0:
        p0 = 1 / (h['beta_0_sigma'] ** 2)
        v = 1 / (p0 + n * yp)
        s = np.sum(y_obs[None, :] - b1[:, None] * x_obs[None, :], axis=1)
        m = (p0 * h['beta_0_mu'] + yp * s) * v
        b0 = m + np.sqrt(v) * z
      else:
        p1 = 1 / (h['beta_1_sigma'] ** 2)
        v = 1 / (p1 + yp * sxx)
        s = np.sum(x_obs[None, :] * (y_obs[None, :] - b0[:, None]), axis=1)
        m = (p1 * h['beta_1_mu'] + yp * s) * v
        b1 = m + np.sqrt(v) * z
    lp = loglik(x_obs, y_obs, b0, b1, ys)
    if vsets is not None:
      with np.errstate(over='ignore'):    # two NEARLY_NEGATIVE_INF -> -inf
        for q in prior_terms((b0, b1, ys), vsets):
          lp = lp + q
    vx[:, t, 0], vx[:, t, 1], vx[:, t, 2] = b0, b1, ys
    vp[:, t] = lp
  return {'v_x': vx, 'v_p': vp}
