"""User-conditional Gibbs for the conjugate linear regression of
examples/mcmc/gibbs_linreg.py, on the GPU.

The reference runs `RF.set_tfun(cond_reg, tsteps=1, x=x_obs, y=y_obs)` on
paras = beta_0 & beta_1 & y_sigma with `SP.set_scores('gibbs')`: each SP.next
calls cond_reg for ONE parameter (rf.py:413-462, cycling through __cond_mod),
accepts it (sp_utils.py:75-84) and evaluates v.prob = the iid sum of
norm.logpdf(y, b0 + b1 x, y_sigma) plus the joint uniform root priors
(rf.py:541-562, rv_utils.py:30-38).

`LinRegConditional` is a plain callable with cond_reg's signature and
NumPy-global draws, so the SAME object runs in the reference as the user tfun;
the façade (`SP.lower`) recognises it and lowers the process to
`pbh_linreg_gibbs` (probayes_amd/csrc/pbh_linreg.hip).  A user's own cond_reg
(the example's closure) is identified by probing (identify_conditional); other
user tfuns raise NotLowerable.  `run` is the batched entry: all chains in one kernel launch.
"""
import ctypes

import numpy as np

from probayes_amd import _lib

_dp = ctypes.POINTER(ctypes.c_double)
KEYS = ('beta_0', 'beta_1', 'y_sigma')


def _ptr(a):
  return None if a is None else a.ctypes.data_as(_dp)


class LinRegConditional:
  """cond_reg of gibbs_linreg.py:34-62 as a descriptor: draws the conditional
  of `unknown` given the others with np.random.gamma / np.random.normal, in
  the reference's arithmetic."""

  def __init__(self, n_obs, beta_0_mu=0., beta_0_sigma=1., beta_1_mu=0.,
               beta_1_sigma=1., y_sigma_alpha=1., y_sigma_beta=1.):
    self.n_obs = int(n_obs)
    self.hyper = (float(beta_0_mu), float(beta_0_sigma), float(beta_1_mu),
                  float(beta_1_sigma), float(y_sigma_alpha),
                  float(y_sigma_beta))

  def __call__(self, x, y, beta_0, beta_1, y_sigma, unknown):
    m0, s0, m1, s1, a, b = self.hyper
    n = self.n_obs
    if unknown == 'y_sigma':
      cond_alpha = a + 0.5 * n
      cond_beta = b + 0.5 * np.sum((y - beta_0 - beta_1 * x) ** 2)
      return 1 / np.sqrt(np.random.gamma(cond_alpha, 1 / cond_beta))
    y_prec = 1 / (y_sigma ** 2)
    if unknown == 'beta_0':
      p0 = 1 / (s0 ** 2)
      cond_var = 1 / (p0 + n * y_prec)
      cond_mu = (p0 * m0 + y_prec * np.sum(y - beta_1 * x)) * cond_var
      return np.random.normal(cond_mu, np.sqrt(cond_var))
    if unknown == 'beta_1':
      p1 = 1 / (s1 ** 2)
      cond_var = 1 / (p1 + y_prec * np.sum(x ** 2))
      cond_mu = (p1 * m1 + y_prec * np.sum(x * (y - beta_0))) * cond_var
      return np.random.normal(cond_mu, np.sqrt(cond_var))
    raise ValueError("Unknown unknown: {}".format(unknown))


def run(x_obs, y_obs, init, n_steps, hyper=(0., 1., 0., 1., 1., 1.),
        vsets=((-6., 6.), (-6., 6.), (0.001, 10.)), rng='philox', seed=0,
        rand=None, step0=0, chain_offset=0, device=0, reps=1, trace=True):
  """Runs N chains for n_steps on the GPU.  init [N, 3] (beta_0, beta_1,
  y_sigma).  rng 'replay' reads rand [n_steps, N] (standard draws in NumPy's
  legacy order); 'philox' (fast sufficient-statistics form) and 'philox_f64'
  (reference arithmetic) draw on the device.  vsets: closed (lo, hi) of the
  joint=True root priors, None for none.  Returns a dict with v_x
  [N, T, 3], v_p [N, T] (when trace), final_x [N, 3], final_p [N] and the
  average kernel ms."""
  x_obs = np.ascontiguousarray(x_obs, np.float64)
  y_obs = np.ascontiguousarray(y_obs, np.float64)
  if x_obs.shape != y_obs.shape or x_obs.ndim != 1:
    raise ValueError('x_obs and y_obs must be 1-D of the same length')
  init = np.asarray(init, np.float64)
  if init.ndim != 2 or init.shape[1] != 3:
    raise ValueError('init must be [N, 3]')
  n = init.shape[0]
  T = int(n_steps)
  mode = _lib.RNG[rng]
  if mode == _lib.RNG['xoshiro']:
    raise ValueError('linreg Gibbs supports replay, philox and philox_f64')
  if mode == _lib.RNG['replay']:
    rand = np.ascontiguousarray(rand, np.float64)
    if rand.shape != (T, n):
      raise ValueError('rand must be [n_steps, N] = {}'.format((T, n)))
  else:
    rand = None
  h = np.asarray(hyper, np.float64)
  v = None if vsets is None else np.asarray(vsets, np.float64).reshape(6)
  init_t = np.ascontiguousarray(init.T)
  tx = np.empty((T, 3, n)) if trace and T else None
  tp = np.empty((T, n)) if trace and T else None
  fx = np.empty((3, n))
  fp = np.full(n, np.nan)
  ms = ctypes.c_double(0.)
  _lib.call('pbh_linreg_gibbs', int(device), len(x_obs), _ptr(x_obs),
            _ptr(y_obs), _ptr(h), _ptr(v), n, int(chain_offset), T,
            int(step0), _ptr(init_t), mode, ctypes.c_uint64(int(seed)),
            _ptr(rand), _ptr(tx), _ptr(tp), _ptr(fx), _ptr(fp), int(reps),
            ctypes.byref(ms))
  out = {'final_x': fx.T.copy(), 'final_p': fp, 'ms': ms.value}
  if tx is not None:
    out['v_x'] = np.transpose(tx, (2, 0, 1)).copy()
    out['v_p'] = tp.T.copy()
  elif trace:   # T == 0: empty traces, as the MH path returns
    out['v_x'] = np.empty((n, 0, 3))
    out['v_p'] = np.empty((n, 0))
  return out


def legacy_streams(n_steps, n_obs, y_sigma_alpha, seeds=None, step0=0):
  """The standard draws the reference's cond_reg consumes, [n_steps, N]:
  standard_gamma(alpha + n/2) on y_sigma steps, gauss otherwise (NumPy's
  legacy normal/gamma = loc + scale * gauss / scale * standard_gamma).  With
  seeds=None: one chain on NumPy's GLOBAL stream, advanced exactly as the
  reference advances it; otherwise one RandomState(seed) per chain."""
  alpha = y_sigma_alpha + 0.5 * n_obs
  gens = [np.random] if seeds is None else \
      [np.random.RandomState(int(s)) for s in seeds]
  out = np.empty((n_steps, len(gens)), np.float64)
  for c, g in enumerate(gens):
    for t in range(n_steps):
      out[t, c] = g.standard_gamma(alpha) if (step0 + t) % 3 == 2 \
          else g.standard_normal()
  return out


class _Recorder:
  """Stands in for np.random.normal / np.random.gamma while a user
  conditional is probed: records the arguments, returns a chosen value."""

  def __init__(self, value):
    self.value, self.calls = value, []

  def __call__(self, *args, **kwds):
    if kwds.get('size') is not None:
      raise ValueError('size= in a conditional draw')
    self.calls.append((args, kwds))
    return self.value


def _probe(fn, x_obs, y_obs, vals, unknown, z=0.6180339887498949,
           g=1.7320508075688772):
  """fn(x, y, **vals, unknown) with NumPy's normal / gamma recorded:
  (draw kind, (loc, scale) or (shape, scale), output, the stub value)."""
  normal, gamma = _Recorder(z), _Recorder(g)
  saved = np.random.normal, np.random.gamma
  np.random.normal, np.random.gamma = normal, gamma
  try:
    out = fn(x=x_obs, y=y_obs, unknown=unknown, **vals)
  finally:
    np.random.normal, np.random.gamma = saved
  if len(normal.calls) + len(gamma.calls) != 1:
    raise ValueError('expected exactly one draw')
  kind, rec = ('normal', normal) if normal.calls else ('gamma', gamma)
  args, kwds = rec.calls[0]
  names = ('loc', 'scale') if kind == 'normal' else ('shape', 'scale')
  full = dict(zip(names, args))
  full.update(kwds)
  return kind, (float(full[names[0]]), float(full.get('scale', 1.))), \
      float(out), rec.value


def _snap(v):
  """A hyper-parameter recovered by probing, rounded to 12 significant
  digits (the user wrote a short literal; verification decides)."""
  return float('{:.12g}'.format(v))


def identify_conditional(fn, x_obs, y_obs, n_probe=4):
  """Hyper-parameters (b0_mu, b0_sigma, b1_mu, b1_sigma, alpha, beta) of a
  user conditional with cond_reg's law (gibbs_linreg.py:34-62), found by
  PROBING it: np.random.normal / gamma are replaced by recorders, the
  callable is run at chosen parameter values, and the draw arguments it
  passes identify the hyper-parameters (at y_sigma = inf the data terms
  vanish: scale = beta_k_sigma, loc = beta_k_mu).  The identified form is
  then verified at random points against LinRegConditional -- draw
  arguments within 1e-12 relative and the output transform (the draw
  itself, or 1 / sqrt(gamma draw)) exact.  Raises NotLowerable otherwise."""
  from probayes_amd.lower import NotLowerable
  x_obs = np.asarray(x_obs, np.float64)
  y_obs = np.asarray(y_obs, np.float64)
  n = len(x_obs)
  try:
    with np.errstate(divide='ignore', invalid='ignore', over='ignore'):
      hyper = []
      for key, other in (('beta_0', 'beta_1'), ('beta_1', 'beta_0')):
        vals = {'beta_0': 0.3, 'beta_1': -0.2, 'y_sigma': np.inf}
        kind, (loc, scale), _, _ = _probe(fn, x_obs, y_obs, vals, key)
        if kind != 'normal':
          raise ValueError('{} must be a normal draw'.format(key))
        hyper += [_snap(loc), _snap(scale)]
      vals = {'beta_0': 0.3, 'beta_1': -0.2, 'y_sigma': 1.}
      kind, (shape, scale), _, _ = _probe(fn, x_obs, y_obs, vals, 'y_sigma')
      if kind != 'gamma':
        raise ValueError('y_sigma must be a gamma draw')
      r = y_obs - 0.3 - -0.2 * x_obs
      hyper += [_snap(shape - 0.5 * n), _snap(1 / scale - 0.5 * np.sum(r ** 2))]
      ref = LinRegConditional(n, *hyper)
      rs = np.random.RandomState(2024)
      for _ in range(n_probe):
        vals = {'beta_0': rs.uniform(-3, 3), 'beta_1': rs.uniform(-3, 3),
                'y_sigma': rs.uniform(0.05, 4.)}
        for key in KEYS:
          got = _probe(fn, x_obs, y_obs, vals, key)
          want = _probe(ref, x_obs, y_obs, vals, key)
          if got[0] != want[0] or got[2] != want[2]:
            raise ValueError('{}: different draw or output transform'.format(key))
          a, b = np.array(got[1]), np.array(want[1])
          if not np.all(np.abs(a - b) <= 1e-12 * np.abs(b)):
            raise ValueError('{}: draw arguments {} != {}'.format(key, a, b))
  except NotLowerable:
    raise
  except Exception as e:   # noqa: BLE001 -- any failure: not this form
    raise NotLowerable('user tfun is not the linear-regression conditional '
                       '(gibbs_linreg.py cond_reg): {}'.format(e))
  if not (hyper[1] > 0 and hyper[3] > 0 and hyper[4] > 0):
    raise NotLowerable('identified hyper-parameters {} are invalid'.format(hyper))
  return tuple(hyper)


def identify_loglik(prob, x_obs, y_obs, n_probe=3):
  """True when the user density equals norm.logpdf(y, b0 + b1 x, y_sigma)
  elementwise (gibbs_linreg.py:31-32) at random parameter points: the
  kernel's v.prob form."""
  import scipy.stats
  rs = np.random.RandomState(12345)
  for _ in range(n_probe):
    b0, b1 = rs.uniform(-3, 3, size=2)
    sg = rs.uniform(0.1, 3.)
    try:
      got = np.asarray(prob(x=x_obs, y=y_obs, beta_0=b0, beta_1=b1,
                            y_sigma=sg), np.float64)
    except Exception:   # noqa: BLE001 -- any failure means "not this form"
      return False
    want = scipy.stats.norm.logpdf(y_obs, loc=b0 + b1 * x_obs, scale=sg)
    if got.shape != want.shape or not np.allclose(got, want, rtol=1e-12,
                                                  atol=1e-12):
      return False
  return True
