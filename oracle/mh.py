"""Vectorised restatement of the reference's MH chain-step (one lane per chain).

Restates, for N independent chains at once, SP.next (sp.py:221-258) with
SD._sample_tran (sd.py:253-288), the proposal forms of Field/Variable
(field.py:469-552, variable.py:600-697), the joint density (rf.py:541-581,
sd.py:148-161, rv_utils.py:8-47) and the hastings/metropolis acceptance
(sp_utils.py:19-64, pscales.py:56-65,100-131,219-236).  Bit-identical per chain
to the reference on the same legacy streams (tests/test_oracle_golden.py).
TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).
"""
import numpy as np
import scipy.stats

# constants.py:9-35 (DEFAULT_FP_PRECISION = 64)
NEARLY_POSITIVE_ZERO = 2.2250738585072014e-308
NEARLY_POSITIVE_INF = 1.7976931348623158e+308
NEARLY_NEGATIVE_INF = -NEARLY_POSITIVE_INF
LOG_NEARLY_POSITIVE_INF = np.log(NEARLY_POSITIVE_INF)


def exp_logp(logp):
  """pscales.py:56-65: exp clamped at LOG_NEARLY_POSITIVE_INF."""
  logp = np.asarray(logp, dtype=np.float64)
  out = np.full(logp.shape, NEARLY_POSITIVE_INF)
  ok = logp <= LOG_NEARLY_POSITIVE_INF
  out[ok] = np.exp(logp[ok])
  return out


def rescale_to_lin(prob, pscale):
  """pscales.py:100-131 rescale(prob, pscale, 1.): identity for a linear
  pscale, exp_logp for a log pscale (d_offs = 0)."""
  return np.asarray(prob, np.float64) if pscale == 'lin' else exp_logp(prob)


def div_prob(dividend, divisor, pscale):
  """pscales.py:219-236 div_prob(a, b, pscale, pscale, pscale=1.)."""
  a = rescale_to_lin(dividend, pscale)
  b = rescale_to_lin(divisor, pscale)
  return a / np.maximum(NEARLY_POSITIVE_ZERO, b)


# ----------------------------------------------------------------------------
# Proposal (delta) forms
# ----------------------------------------------------------------------------
def eval_delta(spec, draws):
  """draws: [R-1 or d, N] of this step's delta randoms -> delta [d, N].

  A covariance-matrix tran (proposal['tfun'], the Cholesky factor that
  RF.set_tran(ndarray) installs, rf.py:210-220) multiplies the base delta of
  every chain: tfun().dot(delta) (rf.py:340-354), one np.dot per chain as the
  reference makes it."""
  delta = _base_delta(spec, draws)
  tf = spec['proposal'].get('tfun')
  if tf is None:
    return delta
  tf = np.asarray(tf, np.float64)
  out = np.empty_like(delta)
  for c in range(delta.shape[1]):
    out[:, c] = tf.dot(np.array(delta[:, c], dtype=float))
  return out


def _base_delta(spec, draws):
  prop, d = spec['proposal'], int(spec['dim'])
  kind = prop['kind']
  if kind == 'gauss':
    # scipy rv_generic.rvs: vals * scale + loc, one call per Delta keyword
    order = np.asarray(prop['order'])
    loc, scale = np.asarray(prop['loc']), np.asarray(prop['scale'])
    delta = np.empty_like(draws[:d])
    for j in range(d):
      k = order[j]
      delta[k] = draws[j] * scale[k] + loc[k]
    return delta
  if kind == 'uniform':
    # variable.py:633 np.random.uniform(-delta, delta) = low + range * u
    dl = np.asarray(prop['delta'])[:, None]
    return -dl + (dl - -dl) * draws[:d]
  if kind == 'sphere':
    # field.py:509-531; delta already multiplied by rss when scale=True
    dl = float(prop['delta'])
    deltas = -dl + (dl - -dl) * draws[:d]
    ss = np.sum(deltas ** 2., axis=0)
    rss = np.zeros_like(ss)
    ok = ss >= NEARLY_POSITIVE_ZERO            # pscales.py real_sqrt
    rss[ok] = np.sqrt(ss[ok])
    deltas = (deltas * dl) / rss
    lengths = np.asarray(prop['lengths'])[:, None]
    return deltas * lengths
  if kind == 'vardelta':
    # per-variable deltas, Variable.eval_delta (variable.py:600-640); the
    # stream holds the (redraw-resolved) uniform, or the randint value
    mode, dl = np.asarray(prop['mode']), np.asarray(prop['delta'])
    delta = np.empty_like(draws[:d])
    for k in range(d):
      if mode[k] == FIXED:
        delta[k] = dl[k]
      elif mode[k] == POLARITY:       # delta if uniform() > 0.5 else -delta
        delta[k] = np.where(draws[k] > 0.5, dl[k], -dl[k])
      elif mode[k] == UNIFORM:        # uniform(-delta, delta)
        delta[k] = -dl[k] + (dl[k] - -dl[k]) * draws[k]
      else:                           # randint(-delta, delta)
        delta[k] = draws[k]
    return delta
  raise ValueError(kind)


# per-variable delta modes of the 'vardelta' proposal (variable.py:600-640)
FIXED, POLARITY, UNIFORM, RANDINT = 0, 1, 2, 3


def apply_delta(spec, x, delta):
  """variable.py:693-739 per chain (scalar values): x + delta, or
  ufun[1](ufun[0](x) + delta); revtype to int for int variables; then, with
  bound=True, a clamp to closed limits, or for an exclusive limit the
  predecessor value (the scalar branch, variable.py:715-728)."""
  prop = spec['proposal']
  vint = prop.get('vint')
  bnd = prop.get('bound')
  out = np.empty_like(x)
  for k in range(int(spec['dim'])):
    if spec['ufun'][k]:
      v = np.exp(np.log(x[k]) + delta[k])
    else:
      v = x[k] + delta[k]
    if vint is not None and vint[k]:
      v = np.trunc(v)                 # vtypes.py:156-166 int(v)
    if bnd is not None and bnd['on'][k]:
      lo, hi = bnd['lo'][k], bnd['hi'][k]
      xl, xh = bnd['xlo'][k], bnd['xhi'][k]
      if not xl and not xh:
        v = np.maximum(lo, np.minimum(hi, v))
      elif xl and xh:
        v = np.where((v > lo) & (v < hi), v, x[k])
      elif xl:
        v = np.where(v < lo, x[k], np.minimum(hi, v))
      else:
        v = np.where(v > hi, x[k], np.maximum(lo, v))
    out[k] = v
  return out


# ----------------------------------------------------------------------------
# Joint density
# ----------------------------------------------------------------------------
def target_prob(spec, x):
  """Density (log or lin per spec['pscale']) of states x [d, N] -> [N]."""
  tg, d = spec['target'], int(spec['dim'])
  kind = tg['kind']
  if kind == 'diag_gauss':
    # user lp(**kw) = sum(norm.logpdf(...)): Python sum, left to right from 0
    mu, sg = np.asarray(tg['mu']), np.asarray(tg['sigma'])
    out = 0
    for i in range(d):
      out = out + scipy.stats.norm.logpdf(x[i], mu[i], sg[i])
    return np.asarray(out, np.float64)
  if kind == 'norm_iid':
    # prob.py:331-380 scipy logpdf over obs, then PD.prod = np.sum (pd.py:368)
    obs = np.asarray(tg['obs'])[None, :]
    loc, scale = x[tg['loc']][:, None], x[tg['scale']][:, None]
    return np.sum(scipy.stats.norm.logpdf(obs, loc=loc, scale=scale), axis=-1)
  if kind == 'gmm':
    logw, mu, sd = np.asarray(tg['logw']), np.asarray(tg['mu']), \
        np.asarray(tg['sd'])
    a = logw[:, None]
    for i in range(d):
      a = a + scipy.stats.norm.logpdf(x[i][None, :], mu[:, i:i + 1],
                                      sd[:, None])
    m = np.max(a, axis=0)
    return m + np.log(np.sum(np.exp(a - m[None, :]), axis=0))
  if kind == 'norm_pdf':
    loc, sc = np.asarray(tg['loc']), np.asarray(tg['scale'])
    out = scipy.stats.norm.pdf(x[0], loc=loc[0], scale=sc[0])
    for i in range(1, d):
      out = out * scipy.stats.norm.pdf(x[i], loc=loc[i], scale=sc[i])
    return np.asarray(out, np.float64)
  if kind == 'uniform_pdf':
    lo, sc = np.asarray(tg['lo']), np.asarray(tg['scale'])
    out = scipy.stats.uniform.pdf(x[0], loc=lo[0], scale=sc[0])
    for i in range(1, d):
      out = out * scipy.stats.uniform.pdf(x[i], loc=lo[i], scale=sc[i])
    return np.asarray(out, np.float64)
  if kind == 'mvn':
    # prob.py:349-358 evaluates at [x_{d-2}, ..., x_0, x_{d-1}] (App. A-4);
    # one call per chain, as the reference makes (BLAS gemv per vector).
    perm = mvn_perm(d)
    mvn = scipy.stats.multivariate_normal(np.asarray(tg['mean']),
                                          np.asarray(tg['cov']))
    shape = (1,) * d + (d,)   # np.stack(np.meshgrid(*vals), axis=-1)
    return np.array([mvn.pdf(x[perm, c].reshape(shape)) for c in
                     range(x.shape[1])], dtype=np.float64).reshape(-1)
  raise ValueError(kind)


def mvn_perm(d):
  """prob.py:354-357: values reversed, then (only for d > 2) rotated by one."""
  rev = list(range(d))[::-1]
  if d > 2:
    rev = rev[1:] + rev[:1]
  return np.array(rev, dtype=np.int64)


def prior_prob(spec, x):
  """joint=True root prior: rv_prod_rule (rf_utils.py:10-42) of uniform_prob
  (rv_utils.py:30-38): logp inside every bound, NEARLY_NEGATIVE_INF outside."""
  pr = spec['prior']
  inside = np.ones(x.shape[1], dtype=bool)
  for i in range(int(spec['dim'])):
    lo_ok = x[i] >= pr['lo'][i] if pr['lo_incl'][i] else x[i] > pr['lo'][i]
    hi_ok = x[i] <= pr['hi'][i] if pr['hi_incl'][i] else x[i] < pr['hi'][i]
    inside &= lo_ok & hi_ok
  return np.where(inside, pr['logp'], NEARLY_NEGATIVE_INF)


def joint_prob(spec, x):
  p = target_prob(spec, x)
  if spec.get('prior') is not None:
    # sd.py:158-161 product(cond_dist, dist) -> prod_rule log-sum
    p = prior_prob(spec, x) + p
  return p


# ----------------------------------------------------------------------------
# Acceptance
# ----------------------------------------------------------------------------
def tran_prob(spec, x, xp):
  """Value of the transition q(x'|x) for the recognised tran forms."""
  tr = spec['tran']
  if tr['kind'] == 'const':
    return np.full(x.shape[1], float(tr['value']))
  order, off = np.asarray(tr['order']), np.asarray(tr['offset'])
  q = None
  for k in order:
    v = scipy.stats.norm.pdf(xp[k], loc=x[k] + off[k], scale=tr['scale'])
    q = v if q is None else q * v
  return q


def scores(spec, lp_pred, lp_succ, x, xp):
  """sp_utils.py:19-64.  Returns (s, s_none) with s_none marking s=None."""
  pscale = spec['pscale']
  n = lp_succ.shape[0]
  if spec['scores'] == 'metropolis':
    s = np.minimum(1., div_prob(lp_succ, lp_pred, pscale))
    return s, np.zeros(n, bool)
  q = rescale_to_lin(tran_prob(spec, x, xp), pscale)     # :52
  none = q <= 0.                                         # :53-54
  if spec['tran']['sym']:
    s = np.minimum(1., div_prob(lp_succ, lp_pred, pscale))   # :56
  else:
    # rf.py:536 reval_tran returns the forward value: r == q (App. A-6)
    r = q
    s = np.minimum(1., div_prob(lp_succ * q, lp_pred * r, pscale))  # :62-64
    s = np.where(r <= 0., 1., s)                         # :60-61
  return np.where(none, np.nan, s), none


def run_mh(spec, init, streams):
  """Runs T steps for N chains.

  init [N, d] initial values (step 1 proposes from them, sp.py:231-232);
  streams [T, R, N] from oracle.streams.legacy_streams (or any replay stream).
  Returns per-step arrays shaped like the golden fixtures ([N, T, ...]).
  """
  d = int(spec['dim'])
  T, R, N = streams.shape
  x = np.ascontiguousarray(np.asarray(init, np.float64).reshape(N, d).T)
  lp = np.zeros(N)
  out = {'v_x': np.empty((N, T, d)), 'v_p': np.empty((N, T)),
         'p_x': np.empty((N, T, d)), 'p_p': np.empty((N, T)),
         's': np.empty((N, T)), 't': np.empty((N, T)),
         'u': np.empty((N, T), np.uint8)}
  for t in range(T):
    draws = streams[t]
    xp = apply_delta(spec, x, eval_delta(spec, draws))
    lpp = joint_prob(spec, xp)
    thr = draws[R - 1]
    if t == 0:
      s, none = np.full(N, np.nan), np.ones(N, bool)   # first step: o is None
    else:
      s, none = scores(spec, lp, lpp, x, xp)
    acc = none | (s >= thr)                            # sp_utils.py:34-37
    x = np.where(acc[None, :], xp, x)
    lp = np.where(acc, lpp, lp)
    out['v_x'][:, t] = x.T
    out['v_p'][:, t] = lp
    out['p_x'][:, t] = xp.T
    out['p_p'][:, t] = lpp
    out['s'][:, t] = s
    out['t'][:, t] = thr
    out['u'][:, t] = acc
  return out
