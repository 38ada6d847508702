"""Vectorised NumPy restatement of the cfg2 chain-step -- TEST / BASELINE
INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg); never imported by the
product path.

The reference's SP.next for the cfg2 model: proposal
x' = x + Delta with Delta_i = norm.rvs(0, 0.5) per dim (the callable delta,
examples/mcmc/mcmc_prob2.py:31 form), joint log-density sum_i
norm.logpdf(x_i, mu_i, sigma_i) (scipy's _norm_logpdf: -y^2/2 - logC -
log sigma), hastings ratio form s = min(1, exp(lp') / max(tiny, exp(lp)))
(sp_utils.py:40-64, pscales.py:219-236) against t = uniform() drawn every
step (sp_utils.py:30-31), step 1 auto-accepted, every step recorded
(sp.py:281-295) -- for N chains at once in [d][N] layout.  Draws come from
NumPy's Generator (PCG64) in bulk rather than per-chain legacy RandomState
streams, so chains are not bit-identical to the reference's
(oracle.run_mh is the bit-exact per-chain restatement); the arithmetic per
chain-step is the same, which is what a CPU throughput baseline measures.
"""
import numpy as np

LOG_C = np.log(np.sqrt(2 * np.pi))
TINY = 2.2250738585072014e-308   # constants.py NEARLY_POSITIVE_ZERO


def cfg2_run(n, t, mu, sigma, step=0.5, seed=0):
  """t chain-steps of n chains; returns (trace_x [t][d][n], trace_lp [t][n],
  trace_u [t][n], final x [d][n])."""
  mu = np.asarray(mu, np.float64)[:, None]
  sigma = np.asarray(sigma, np.float64)[:, None]
  logs = np.log(sigma)
  d = mu.shape[0]
  rng = np.random.Generator(np.random.PCG64(seed))
  x = np.zeros((d, n))
  lp = np.zeros(n)
  tx = np.empty((t, d, n))
  tl = np.empty((t, n))
  tu = np.empty((t, n), bool)
  for s in range(t):
    xp = x + step * rng.standard_normal((d, n))
    y = (xp - mu) / sigma
    lpp = np.sum(-(y * y) / 2.0 - LOG_C - logs, axis=0)
    u = rng.random(n)
    if s == 0:
      acc = np.ones(n, bool)
    else:
      with np.errstate(over='ignore', under='ignore'):
        r = np.minimum(1.0, np.exp(lpp) / np.maximum(TINY, np.exp(lp)))
      acc = r >= u
    x = np.where(acc, xp, x)
    lp = np.where(acc, lpp, lp)
    tx[s] = x
    tl[s] = lp
    tu[s] = acc
  return tx, tl, tu, x
