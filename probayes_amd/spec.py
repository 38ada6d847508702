"""Plain-data workload spec: the lowered form of an SP model.

A spec is a dict of numbers and arrays (no code).  The SP facade lowers a
recognised model to it, probayes_amd.engine packs it into the C-ABI structs of
include/pbhip.h, and the tests hand the very same dict to the CPU oracle.  It
encodes the closed set of model forms the engine lowers:

  target  kind  diag_gauss  sum_i norm.logpdf(x_i, mu_i, sigma_i)  (log)
                norm_iid    sum_obs norm.logpdf(obs, x[loc], x[scale]) (log, iid)
                gmm         logsumexp_k(logw_k + sum_i norm.logpdf(x_i, mu_ki, sd_k)) (log)
                norm_pdf    prod_i norm.pdf(x_i, loc_i, scale_i)  (lin)
                uniform_pdf prod_i uniform.pdf(x_i, lo_i, scale_i) (lin)
                mvn         multivariate_normal.pdf at the permuted vector (lin)
  prior         joint=True uniform prior of the root RVs (rv_utils.py:8-47)
  ufun          per-dim 1 = (log, exp) change of variable (variable.py:693-697)
  proposal kind gauss   callable Delta(norm.rvs(loc, scale)) per dim
                sphere  tuple delta (field.py:509-531)
                uniform list delta (variable.py:625-633)
                vardelta per-variable modes (fixed 0 | polarity 1 | uniform 2 |
                        randint 3) and steps: a Delta of containers or a bare
                        scalar Field delta (field.py:266-306, variable.py:600-640)
                (any MH kind may carry vint [d]: int variables, truncated,
                 and bound {on, lo, hi, xlo, xhi}: bound=True, variable.py:700-739)
                (any of the three may carry tfun [d, d]: the covariance
                random walk delta' = tfun . delta, rf.py:210-220, 340-354)
                gibbs   CondCov conditional sampling (cond_cov.py:22-65)
  tran     kind const (value) | gauss_pdf (scale, offset, order); sym flag
  scores        hastings | metropolis | gibbs (sp_utils.py:87-91)
"""
import numpy as np

TARGETS = ('diag_gauss', 'norm_iid', 'gmm', 'norm_pdf', 'uniform_pdf', 'mvn')
PROPOSALS = ('gauss', 'sphere', 'uniform', 'gibbs', 'vardelta')
SCORES = ('hastings', 'metropolis', 'gibbs')


def _vec(v, d, name):
  a = np.asarray(v, dtype=np.float64).reshape(-1)
  if a.size == 1 and d > 1:
    a = np.repeat(a, d)
  if a.size != d:
    raise ValueError('{} must have {} entries, got {}'.format(name, d, a.size))
  return a


def make_spec(dim, target, proposal, scores='hastings', pscale=None,
              tran=None, prior=None, ufun=None, names=None):
  """Validates and normalises a workload spec (all arrays float64)."""
  d = int(dim)
  if d < 1:
    raise ValueError('dim must be >= 1')
  target = dict(target)
  proposal = dict(proposal)
  if target['kind'] not in TARGETS:
    raise ValueError('unknown target kind {}'.format(target['kind']))
  if proposal['kind'] not in PROPOSALS:
    raise ValueError('unknown proposal kind {}'.format(proposal['kind']))
  if scores not in SCORES:
    raise ValueError('unknown scores {}'.format(scores))
  if (scores == 'gibbs') != (proposal['kind'] == 'gibbs'):
    raise ValueError('gibbs scores require the gibbs proposal and vice versa')
  kind = target['kind']
  if pscale is None:
    pscale = 'log' if kind in ('diag_gauss', 'norm_iid', 'gmm') else 'lin'
  if pscale not in ('log', 'lin'):
    raise ValueError('pscale must be log or lin')
  if kind == 'diag_gauss':
    target['mu'] = _vec(target['mu'], d, 'mu')
    target['sigma'] = _vec(target['sigma'], d, 'sigma')
  elif kind == 'norm_iid':
    target['obs'] = np.asarray(target['obs'], dtype=np.float64).reshape(-1)
    target['loc'] = int(target.get('loc', 0))
    target['scale'] = int(target.get('scale', 1))
  elif kind == 'gmm':
    target['logw'] = np.asarray(target['logw'], dtype=np.float64).reshape(-1)
    k = target['logw'].size
    target['mu'] = np.asarray(target['mu'], dtype=np.float64).reshape(k, d)
    target['sd'] = np.asarray(target['sd'], dtype=np.float64).reshape(k)
  elif kind == 'norm_pdf':
    target['loc'] = _vec(target['loc'], d, 'loc')
    target['scale'] = _vec(target['scale'], d, 'scale')
  elif kind == 'uniform_pdf':
    target['lo'] = _vec(target['lo'], d, 'lo')
    target['scale'] = _vec(target['scale'], d, 'scale')
  elif kind == 'mvn':
    target['mean'] = _vec(target['mean'], d, 'mean')
    target['cov'] = np.asarray(target['cov'], dtype=np.float64).reshape(d, d)
  if prior is not None:
    prior = dict(prior)
    prior['lo'] = _vec(prior['lo'], d, 'prior.lo')
    prior['hi'] = _vec(prior['hi'], d, 'prior.hi')
    prior['lo_incl'] = np.asarray(prior.get('lo_incl', [1] * d), dtype=np.int32)
    prior['hi_incl'] = np.asarray(prior.get('hi_incl', [1] * d), dtype=np.int32)
    prior['logp'] = float(prior['logp'])
  ufun = np.zeros(d, np.int32) if ufun is None else \
      np.asarray(ufun, dtype=np.int32).reshape(d)
  pk = proposal['kind']
  if pk == 'gauss':
    proposal['loc'] = _vec(proposal.get('loc', 0.), d, 'loc')
    proposal['scale'] = _vec(proposal['scale'], d, 'scale')
    proposal['order'] = np.asarray(proposal.get('order', range(d)), np.int32)
  elif pk == 'sphere':
    proposal['delta'] = float(proposal['delta'])
    proposal['lengths'] = _vec(proposal.get('lengths', 1.), d, 'lengths')
  elif pk == 'uniform':
    proposal['delta'] = _vec(proposal['delta'], d, 'delta')
  elif pk == 'vardelta':
    proposal['delta'] = _vec(proposal['delta'], d, 'delta')
    proposal['mode'] = np.asarray(proposal['mode'], np.int32).reshape(d)
    if np.any((proposal['mode'] < 0) | (proposal['mode'] > 3)):
      raise ValueError('vardelta modes are 0..3')
  elif pk == 'gibbs':
    proposal['mean'] = _vec(proposal['mean'], d, 'mean')
    proposal['cov'] = np.asarray(proposal['cov'], np.float64).reshape(d, d)
    proposal['lo'] = _vec(proposal['lo'], d, 'lo')
    proposal['hi'] = _vec(proposal['hi'], d, 'hi')
    proposal['tsteps'] = int(proposal.get('tsteps', 1))
  if proposal.get('tfun') is not None:
    if pk == 'gibbs':
      raise ValueError('tfun applies to MH deltas, not to gibbs')
    tf = np.array(proposal['tfun'], dtype=np.float64)
    if tf.shape != (d, d) or not np.all(np.isfinite(tf)):
      raise ValueError('tfun must be a finite [{0}, {0}] matrix'.format(d))
    proposal['tfun'] = tf
  if pk != 'gibbs':
    if proposal.get('vint') is not None:
      proposal['vint'] = np.asarray(proposal['vint'], np.int32).reshape(d)
    if proposal.get('bound') is not None:
      b = dict(proposal['bound'])
      b['lo'], b['hi'] = _vec(b['lo'], d, 'bound.lo'), _vec(b['hi'], d, 'bound.hi')
      for key in ('on', 'xlo', 'xhi'):
        b[key] = np.asarray(b.get(key, [1 if key == 'on' else 0] * d),
                            np.int32).reshape(d)
      proposal['bound'] = b
  if tran is None:
    tran = {'kind': 'const', 'value': 1.0, 'sym': True}
  tran = dict(tran)
  tran.setdefault('sym', True)
  if tran['kind'] == 'gauss_pdf':
    tran['scale'] = float(tran['scale'])
    tran['offset'] = _vec(tran.get('offset', 0.), d, 'offset')
    tran['order'] = np.asarray(tran.get('order', range(d)), np.int32)
  elif tran['kind'] == 'const':
    tran['value'] = float(tran['value'])
  else:
    raise ValueError('unknown tran kind {}'.format(tran['kind']))
  names = list(names) if names is not None else \
      ['x{}'.format(i) for i in range(d)]
  return {'dim': d, 'names': names, 'pscale': pscale, 'target': target,
          'prior': prior, 'ufun': ufun, 'proposal': proposal, 'tran': tran,
          'scores': scores}


def normalize_spec(spec):
  """Re-validates a spec dict (e.g. one built by hand in a test)."""
  keys = ('dim', 'target', 'proposal', 'scores', 'pscale', 'tran', 'prior',
          'ufun', 'names')
  return make_spec(**{k: spec[k] for k in keys if k in spec})
