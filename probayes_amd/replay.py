"""Reference-compatible random streams for the engine's REPLAY mode.

The reference draws every random number from NumPy's legacy RandomState in a
fixed per-step order (sp.py:249, field.py:516,
variable.py:633, mcmc_prob2.py:31, cond_cov.py:57-59).  Feeding the kernels
the same numbers in that order reproduces the reference's chains:
  * single chain, global state: drawn from np.random's global RandomState,
    which the reference itself uses -- after sampling, the global state has
    advanced exactly as the reference would have left it;
  * batched chains: chain c drawn from np.random.RandomState(seeds[c]).
Layout [T][R][N] float64: R = d + 1 (delta draws in the callable's draw order,
then the threshold) for MH, tsteps for CondCov Gibbs.  Normals are stored as
standard normals z, uniforms as the raw random_sample double.
"""
import numpy as np


def _fill(rs, kind, d, tsteps, n_coords, col, var=None):
  """Fills col [T, R] from RandomState rs.  var = (modes, steps) of a
  VARDELTA proposal: per variable in key order a randint value, a raw
  uniform, or nothing for a fixed step (variable.py:618-633)."""
  T = col.shape[0]
  if kind == 'gibbs':
    col[:] = np.nan
    for t in range(T):
      m = n_coords[t]
      col[t, :m] = rs.random_sample(m)
    return
  if kind == 'vardelta':
    modes, steps = var
    col[:, :d] = np.nan
    for t in range(T):
      for k in range(d):
        if modes[k] == 3:
          col[t, k] = rs.randint(-steps[k], steps[k])
        elif modes[k] != 0:
          col[t, k] = rs.random_sample()
      col[t, d] = rs.random_sample()
    return
  for t in range(T):
    if kind == 'gauss':
      col[t, :d] = rs.standard_normal(d)
    else:
      col[t, :d] = rs.random_sample(d)
    col[t, d] = rs.random_sample()


def gibbs_coords_per_step(d, tsteps, T, step0=0):
  """Coordinates updated per SP step (rf.py:446-452 cycling)."""
  nblk = -(-d // tsteps)
  out = np.empty(T, np.int64)
  for t in range(T):
    cm = ((step0 + t) % nblk) * tsteps
    out[t] = min(cm + tsteps, d) - cm
  return out


def stream_width(spec):
  if spec['proposal']['kind'] == 'gibbs':
    return int(spec['proposal'].get('tsteps', 1))
  return int(spec['dim']) + 1


def _chunk(args):
  spec, n_steps, seeds, step0 = args
  return legacy_streams(spec, n_steps, seeds, step0)


def legacy_streams_parallel(spec, n_steps, seeds, processes=8, step0=0):
  """legacy_streams over a process pool (chains are independent); used to
  feed full-size replay runs (65 536 chains) in seconds."""
  import multiprocessing as mp
  seeds = np.asarray(seeds).reshape(-1)
  chunks = np.array_split(seeds, max(1, min(processes, seeds.size)))
  with mp.get_context('fork').Pool(len(chunks)) as pool:
    parts = pool.map(_chunk, [(spec, n_steps, c, step0) for c in chunks])
  return np.concatenate(parts, axis=2)


def legacy_streams(spec, n_steps, seeds=None, step0=0):
  """[T, R, N] streams; seeds=None draws ONE chain from the global state."""
  d, kind = int(spec['dim']), spec['proposal']['kind']
  tsteps = int(spec['proposal'].get('tsteps', 1)) if kind == 'gibbs' else 1
  coords = gibbs_coords_per_step(d, tsteps, n_steps, step0) \
      if kind == 'gibbs' else None
  r = stream_width(spec)
  var = (np.asarray(spec['proposal']['mode']),
         np.asarray(spec['proposal']['delta'], np.float64)) \
      if kind == 'vardelta' else None
  if seeds is None:
    out = np.empty((n_steps, r, 1))
    col = np.empty((n_steps, r))
    _fill(np.random.mtrand._rand, kind, d, tsteps, coords, col, var)
    out[:, :, 0] = col
    return out
  seeds = np.asarray(seeds).reshape(-1)
  out = np.empty((n_steps, r, seeds.size))
  col = np.empty((n_steps, r))
  for c, s in enumerate(seeds):
    _fill(np.random.RandomState(int(s)), kind, d, tsteps, coords, col, var)
    out[:, :, c] = col
  return out
