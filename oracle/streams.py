"""Legacy-MT19937 random streams in the reference's per-step consumption order.

The reference draws every random number from NumPy's global legacy RandomState
(SURVEY.md App. A-7).  Per chain-step, in order:
  gauss proposal (callable Delta of norm.rvs, e.g. examples/mcmc/mcmc_prob2.py:31):
      d x standard_normal (scipy norm.rvs = loc + scale*z), in Delta keyword order
  sphere proposal (tuple delta, field.py:516):   uniform(size=d)  -> d raw doubles
  uniform proposal (list delta, variable.py:633): d x uniform     -> d raw doubles
  then 1 x random_sample for the MH threshold t (sp_utils.py:30-31, sp.py:249)
  gibbs (cond_cov.py:57-59 via vtypes.py:185-186): 1 x random_sample, no threshold.
Standard normals are stored as z; uniforms as the raw random_sample double u in
[0, 1) (numpy's legacy uniform(lo, hi) is lo + (hi - lo) * u).

Layout: [T][R][N] float64 (step, draw, chain) -- the replay layout the engine
reads (chain index fastest, so a wavefront's loads coalesce).
"""
import numpy as np


def stream_width(spec):
  """Draws per chain-step R: d + 1 for MH, tsteps (one
  uniform per updated coordinate, rf.py:446-458) for Gibbs."""
  if spec['proposal']['kind'] == 'gibbs':
    return int(spec['proposal'].get('tsteps', 1))
  return int(spec['dim']) + 1


def gibbs_coords(d, tsteps, n_steps):
  """Coordinates per SP step under the per-RF cycling of rf.py:446-452."""
  out, cm = [], 0
  for _ in range(n_steps):
    out.append(list(range(cm, min(cm + tsteps, d))))
    cm += tsteps
    if cm >= d:
      cm = 0
  return out


def legacy_streams(spec, seeds, n_steps, states=None):
  """Per-chain np.random.RandomState(seed) streams, shape [T, R, N].
  states: a list that receives each chain's RandomState after the draws."""
  seeds = np.asarray(seeds).reshape(-1)
  n, d, r = seeds.size, int(spec['dim']), stream_width(spec)
  kind = spec['proposal']['kind']
  out = np.empty((n_steps, r, n), dtype=np.float64)
  for c, seed in enumerate(seeds):
    rs = np.random.RandomState(int(seed))
    if states is not None:
      states.append(rs)
    col = out[:, :, c]
    if kind == 'gibbs':
      col[:] = np.nan
      for t, keys in enumerate(gibbs_coords(d, r, n_steps)):
        col[t, :len(keys)] = rs.random_sample(len(keys))
      continue
    for t in range(n_steps):
      if kind == 'gauss':
        # d separate norm.rvs calls == one standard_normal(d): the polar
        # method's cached second deviate persists across calls either way.
        col[t, :d] = rs.standard_normal(d)
      elif kind in ('uniform', 'vardelta'):
        _per_variable_draws(rs, spec['proposal'], d, col[t])
      else:
        col[t, :d] = rs.random_sample(d)
      col[t, d] = rs.random_sample()
  return out


def _per_variable_draws(rs, prop, d, row):
  """Field.eval_delta draws every variable's delta in key order
  (field.py:477-483, variable.py:618-633): tuple -> uniform() for the
  polarity, list -> uniform(-d, d) or, for an int variable, randint(-d, d),
  bare scalar -> nothing.  Each value comes back wrapped in the variable's
  Delta namedtuple, so apply_delta's `delta or self._delta`
  (variable.py:660) never redraws, not even a zero.  row[k] keeps the raw
  uniform, or the randint value; NaN for a fixed step."""
  from oracle.mh import FIXED, RANDINT
  mode = np.full(d, 2) if prop['kind'] == 'uniform' else np.asarray(prop['mode'])
  dl = np.asarray(prop['delta'], np.float64)
  row[:d] = np.nan
  for k in range(d):
    if mode[k] == RANDINT:
      row[k] = rs.randint(-dl[k], dl[k])
    elif mode[k] != FIXED:
      row[k] = rs.random_sample()
