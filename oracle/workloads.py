"""Specs of the golden workloads (tools/gen_golden.py) as plain dicts.

Each builder restates, in the spec vocabulary of probayes_amd/spec.py, the
reference model that tools/gen_golden.py ran (cited per entry).  The dicts are
complete (every key the engine reads), so tests hand them unchanged to the
oracle and to the engine.  TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).
"""
import json
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))), 'tests', 'golden')

NEARLY_NEGATIVE_INF = -1.7976931348623158e+308


def load_golden(name):
  with np.load(os.path.join(GOLDEN_DIR, name + '.npz'),
               allow_pickle=False) as z:
    g = {k: z[k] for k in z.files}
  g['meta'] = json.loads(str(g['meta']))
  return g


def _spec(dim, names, target, proposal, scores='hastings', pscale='log',
          tran=None, prior=None, ufun=None):
  d = dim
  return {'dim': d, 'names': list(names), 'pscale': pscale, 'target': target,
          'proposal': proposal, 'scores': scores,
          'tran': tran or {'kind': 'const', 'value': 1.0, 'sym': True},
          'prior': prior,
          'ufun': np.zeros(d, np.int32) if ufun is None else
                  np.asarray(ufun, np.int32)}


def _gauss(d, scale, loc=0., order=None):
  return {'kind': 'gauss', 'loc': np.broadcast_to(np.float64(loc), (d,)).copy()
          if np.ndim(loc) == 0 else np.asarray(loc, np.float64),
          'scale': np.full(d, float(scale)),
          'order': np.arange(d, dtype=np.int32) if order is None else
                   np.asarray(order, np.int32)}


def _qpdf(d, scale, order, offset=None, sym=True):
  return {'kind': 'gauss_pdf', 'scale': float(scale), 'sym': sym,
          'order': np.asarray(order, np.int32),
          'offset': np.zeros(d) if offset is None else
                    np.asarray(offset, np.float64)}


def spec_metrohast_norm1d(params):
  """examples/mcmc/metrohast_norm1d.py:22-35: mu in [40,60], sigma in [5,20]
  with (log, exp) ufun; tuple delta (0.005,) scale=True; tran (1., 1.) tuple;
  joint=True uniform root prior, iid obs."""
  mu_len = 60. - 40.
  ul = np.log(np.array([5., 20.]))                  # variable.py:332-335
  sg_len = max(ul) - min(ul)
  lengths = np.array([mu_len, sg_len])
  rss = np.sqrt(np.sum(lengths ** 2))               # field.py:513-515
  prior_logp = -np.log(mu_len) + -np.log(sg_len)    # rv.py:160, rf_utils.py:10-42
  return _spec(2, ['mu', 'sigma'],
               {'kind': 'norm_iid', 'obs': params['x_obs'], 'loc': 0,
                'scale': 1},
               {'kind': 'sphere', 'delta': 0.005 * rss, 'lengths': lengths},
               tran={'kind': 'const', 'value': 1.0, 'sym': False},
               # tuple vsets (40, 60), (5, 20.): both limits exclusive
               # (variable.py:178-183, 360-366)
               prior={'lo': np.array([40., 5.]), 'hi': np.array([60., 20.]),
                      'lo_incl': np.array([0, 0], np.int32),
                      'hi_incl': np.array([0, 0], np.int32),
                      'logp': float(prior_logp)},
               ufun=[0, 1])


def spec_mcmc_prob2(params):
  """examples/mcmc/mcmc_prob2.py:24-31."""
  return _spec(1, ['x'], {'kind': 'norm_pdf', 'loc': np.array([2.]),
                          'scale': np.array([np.sqrt(2)])},
               _gauss(1, 1.), pscale='lin', tran=_qpdf(1, 1., [0]))


def spec_mcmc_prob3(params):
  """examples/mcmc/mcmc_prob3.py:32-39."""
  return _spec(1, ['x'], {'kind': 'uniform_pdf', 'lo': np.array([3.]),
                          'scale': np.array([4.])},
               _gauss(1, 1.), pscale='lin', tran=_qpdf(1, 1., [0]))


_COV4 = np.array([[2.0, 1.2], [1.2, 2.0]])


def spec_mcmc_prob4a(params):
  """examples/mcmc/mcmc_prob4a.py:37-48 (q multiplies the y pdf first)."""
  return _spec(2, ['x', 'y'], {'kind': 'mvn', 'mean': np.zeros(2),
                               'cov': _COV4},
               _gauss(2, 1.), pscale='lin', tran=_qpdf(2, 1., [1, 0]))


def spec_mcmc_prob4b(params):
  """examples/mcmc/mcmc_prob4b.py:34-51."""
  return _spec(2, ['x', 'y'], {'kind': 'uniform_pdf', 'lo': np.array([3., 1.]),
                               'scale': np.array([4., 8.])},
               _gauss(2, 1.), pscale='lin', tran=_qpdf(2, 1., [1, 0]))


def spec_mcmc_prob6(params):
  """examples/mcmc/mcmc_prob6.py:48-61: tran (q, r) tuple -> asymmetric, but
  reval_tran returns q (rf.py:536), delta loc (-2, 0)."""
  return _spec(2, ['x', 'y'], {'kind': 'mvn', 'mean': np.zeros(2),
                               'cov': _COV4},
               _gauss(2, 1., loc=[-2., 0.]), pscale='lin',
               tran=_qpdf(2, 1., [1, 0], offset=[2., 0.], sym=False))


def _gibbs(mean, cov, lo, hi, names):
  d = len(mean)
  return _spec(d, names, {'kind': 'mvn', 'mean': np.asarray(mean, np.float64),
                          'cov': np.asarray(cov, np.float64)},
               {'kind': 'gibbs', 'mean': np.asarray(mean, np.float64),
                'cov': np.asarray(cov, np.float64),
                'lo': np.full(d, float(lo)), 'hi': np.full(d, float(hi)),
                'tsteps': 1},
               scores='gibbs', pscale='lin')


def spec_gibbs_norm2d(params):
  """examples/mcmc/gibbs_norm2d.py:9-19."""
  return _gibbs([0.5, -0.5], [[1.5, -1.0], [-1.0, 2.]], -10., 10., ['x', 'y'])


def spec_gibbs8(params):
  """SURVEY App. B H4 (cfg3 shape)."""
  return _gibbs(params['mean'], params['cov'], -20., 20.,
                ['x{}'.format(i) for i in range(8)])


def spec_gibbs_sweep2(params):
  """examples/cov/multinorm_rw.py model: CondCov tran without tsteps (every
  coordinate per step)."""
  sp = _gibbs([0.5, -0.5], [[1.5, -1.0], [-1.0, 2.]], -10., 10., ['x', 'y'])
  sp['proposal']['tsteps'] = 2
  return sp


def spec_diag10(params):
  """SURVEY App. B H3 (cfg2 shape)."""
  d = len(params['mu'])
  return _spec(d, ['x{}'.format(i) for i in range(d)],
               {'kind': 'diag_gauss', 'mu': np.asarray(params['mu'], float),
                'sigma': np.asarray(params['sigma'], float)},
               _gauss(d, float(params['step'])))


def spec_gmm2(params):
  """SURVEY App. B H5 (cfg5 shape)."""
  return _spec(2, ['x', 'y'],
               {'kind': 'gmm', 'logw': np.log(np.asarray(params['w'], float)),
                'mu': np.asarray(params['mu'], float),
                'sd': np.asarray(params['sd'], float)},
               _gauss(2, float(params['step'])))


def spec_covrw2(params):
  """examples/cov/multinorm_rw.py:6-15 model with a covariance RW proposal
  (tests/mcmc_examples.py covrw2): mvn target, callable N(0, step^2) Delta,
  tfun = chol(cov) (rf.py:210-220, 340-354).  The non-callable tran evaluates
  to the default conditional 1. of the RF's linear pscale (rf.py:20,510-511);
  the subfield route (sd.py:97-105) leaves the SP's _sym_tran False
  (rf.py:179), so hastings takes the reverse branch with r = q (rf.py:536):
  q~ = r~ = rescale(1., pscale) -- e under a log pscale (App. A-1)."""
  cov = np.array([[1.5, -1.0], [-1.0, 2.]])
  prop = _gauss(2, float(params['step']))
  prop['tfun'] = np.linalg.cholesky(cov)
  return _spec(2, ['x', 'y'], {'kind': 'mvn', 'mean': np.array([0.5, -0.5]),
                               'cov': cov}, prop, pscale='lin',
               tran={'kind': 'const', 'value': 1.0, 'sym': False})


def spec_covrw5(params):
  """tests/mcmc_examples.py covrw5: 5-dim diagonal Gaussian, spherical tuple
  delta times chol(cov); tran as spec_covrw2 (e-tempered: log pscale)."""
  d = len(params['mu'])
  return _spec(d, ['x{}'.format(i) for i in range(d)],
               {'kind': 'diag_gauss', 'mu': np.asarray(params['mu'], float),
                'sigma': np.asarray(params['sigma'], float)},
               {'kind': 'sphere', 'delta': float(params['step']),
                'lengths': np.ones(d),
                'tfun': np.linalg.cholesky(np.asarray(params['cov'], float))},
               tran={'kind': 'const', 'value': 1.0, 'sym': False})


# ----------------------------------------------------------------------------
# Delta forms (tests/mcmc_examples.py DELTA_WORKLOADS): per-variable modes
# FIXED / POLARITY / UNIFORM / RANDINT (oracle.mh), int truncation and the
# bound=True clamp / bounce of variable.py:700-739.
# ----------------------------------------------------------------------------
def _bound(lo, hi, xlo, xhi, on=None):
  d = len(lo)
  return {'lo': np.asarray(lo, np.float64), 'hi': np.asarray(hi, np.float64),
          'xlo': np.asarray(xlo, np.int32), 'xhi': np.asarray(xhi, np.int32),
          'on': np.ones(d, np.int32) if on is None else np.asarray(on, np.int32)}


def _diag(mu, sigma):
  return {'kind': 'diag_gauss', 'mu': np.asarray(mu, np.float64),
          'sigma': np.asarray(sigma, np.float64)}


# x [(-1,), 1], y [-1, (1,)], z [0, 2] (tests/mcmc_examples.py _three_vsets)
_B3 = _bound([-1., -1., 0.], [1., 1., 2.], [1, 0, 0], [0, 1, 0])
_T3 = _diag([-0.8, 0.8, 1.9], [0.5, 0.5, 0.6])


def spec_bound_sphere2(params):
  """omc_rw_circle.py:16-22: tuple vsets = both limits exclusive
  (variable.py:178-183), unscaled spherical delta, bound=True bounces."""
  prop = {'kind': 'sphere', 'delta': float(params['step']),
          'lengths': np.ones(2), 'bound': _bound([-1., -1.], [1., 1.],
                                                 [1, 1], [1, 1])}
  return _spec(2, ['x', 'y'], _diag([0.7, -0.6], [0.4, 0.5]), prop)


def spec_bound_list3(params):
  """set_delta([0.2], {'z': 0.15}, scale=True, bound=True): x, y uniform
  +-0.2 * length 2, z +-0.15 unscaled (field.py:276-306)."""
  prop = {'kind': 'uniform', 'delta': np.array([0.2 * 2., 0.2 * 2., 0.15]),
          'bound': _B3}
  return _spec(3, ['x', 'y', 'z'], _T3, prop)


def spec_pervar3(params):
  """Delta(x=(0.25,), y=[0.3], z=0.05), scale=True: only the bare scalar is
  scaled by its length (variable.py:637-639)."""
  prop = {'kind': 'vardelta', 'mode': np.array([1, 2, 0], np.int32),
          'delta': np.array([0.25, 0.3, 0.05 * 2.]), 'bound': _B3}
  return _spec(3, ['x', 'y', 'z'], _T3, prop)


def spec_dict3(params):
  """A dict delta leaves every value unchanged (tests/mcmc_examples.py dict3):
  fixed zero steps, no bound (apply_delta returns before bounding)."""
  prop = {'kind': 'vardelta', 'mode': np.zeros(3, np.int32),
          'delta': np.zeros(3)}
  return _spec(3, ['x', 'y', 'z'], _T3, prop)


def spec_fixed2(params):
  """set_delta(0.02, {'y': -0.03}, scale=True, bound=True) on [-1, 1]^2."""
  prop = {'kind': 'vardelta', 'mode': np.zeros(2, np.int32),
          'delta': np.array([0.02 * 2., -0.03]),
          'bound': _bound([-1., -1.], [1., 1.], [0, 0], [0, 0])}
  return _spec(2, ['x', 'y'], _diag([0.3, -0.2], [0.5, 0.4]), prop)


def spec_randint2(params):
  """Delta(n=[3], x=[0.5]), bound=True: n int in range(0, 21) draws
  randint(-3, 3) and clamps to [0, 20]; x's tuple vset (-inf, inf) bounces
  only non-finite values."""
  prop = {'kind': 'vardelta', 'mode': np.array([3, 2], np.int32),
          'delta': np.array([3., 0.5]), 'vint': np.array([1, 0], np.int32),
          'bound': _bound([0., -np.inf], [20., np.inf], [0, 1], [0, 1])}
  return _spec(2, ['n', 'x'], _diag([12., 0.], [3., 1.]), prop)


INITS = {
    'metrohast_norm1d': [50., 12.5], 'mcmc_prob2': [0.], 'mcmc_prob3': [5.],
    'mcmc_prob4a': [0., 1.], 'mcmc_prob4b': [5., 5.], 'mcmc_prob6': [0., 1.],
    'gibbs_norm2d': [0., 1.], 'diag10': [0.] * 10, 'gibbs8': [0.] * 8,
    'gibbs_sweep2': [0., 0.],
    'gmm2': [0., 0.], 'covrw2': [0., 0.], 'covrw5': [0.] * 5,
    'bound_sphere2': [0., 0.], 'bound_list3': [0., 0., 1.],
    'pervar3': [0., 0., 1.], 'dict3': [0.1, 0.2, 1.], 'fixed2': [0., 0.],
    'randint2': [0., 0.],
}

WORKLOADS = {
    'metrohast_norm1d': spec_metrohast_norm1d, 'mcmc_prob2': spec_mcmc_prob2,
    'mcmc_prob3': spec_mcmc_prob3, 'mcmc_prob4a': spec_mcmc_prob4a,
    'mcmc_prob4b': spec_mcmc_prob4b, 'mcmc_prob6': spec_mcmc_prob6,
    'gibbs_norm2d': spec_gibbs_norm2d, 'diag10': spec_diag10,
    'gibbs8': spec_gibbs8, 'gmm2': spec_gmm2,
    'gibbs_sweep2': spec_gibbs_sweep2,
    'covrw2': spec_covrw2, 'covrw5': spec_covrw5,
    'bound_sphere2': spec_bound_sphere2, 'bound_list3': spec_bound_list3,
    'pervar3': spec_pervar3, 'dict3': spec_dict3, 'fixed2': spec_fixed2,
    'randint2': spec_randint2,
}

# consecutive samplers on one process (tests/mcmc_examples.py SEGMENTED)
SEGMENTED = {'gibbs_norm2d_seg': 'gibbs_norm2d',
             'gibbs_linreg_seg': 'gibbs_linreg'}


def golden_params(g):
  return {k[len('param_'):]: v for k, v in g.items() if k.startswith('param_')}


def golden_spec(name, g=None):
  g = load_golden(name) if g is None else g
  return WORKLOADS[name](golden_params(g))


def golden_init(name, n):
  return np.tile(np.asarray(INITS[name], np.float64), (n, 1))
