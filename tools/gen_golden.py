"""Golden-vector generator: runs the REFERENCE probayes (this container only).

This script imports the reference package from /root/reference to record chain
traces that pin the oracle (oracle/) and, through it, the HIP engine.  It never
runs on the GPU box and nothing in tests/, bench.py or __graft_entry__ imports it.

Recipe:
    mkdir -p /tmp/stub && echo '' > /tmp/stub/h5py.py
    PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg PYTHONPATH=/tmp/stub:/root/reference \
        python3 tools/gen_golden.py [names...]

Each workload runs on a FRESH SP instance per chain (the reference keeps
__last/__counter per sampler and __cond_mod per RF: sp.py:26-28, rf.py:446-452)
with the global NumPy RandomState re-seeded by np.random.seed(seed0 + chain).
The model builders restate examples/mcmc/*.py (cited per builder) with only the
step counts and seeds changed.

Output: tests/golden/<name>.npz holding inputs (seeds, init, model params) and
expected outputs per chain/step:
    v_x[c, t, k]  accepted state after step t (summary.v[key])      sp.py:253-256
    v_p[c, t]     its (log-)probability (summary.v.prob)
    p_x[c, t, k]  proposed state (opqr.p values)                     sd.py:280-288
    p_p[c, t]     proposed (log-)probability
    s[c, t]       MH score (nan when None)                            sp_utils.py:40-64
    t[c, t]       threshold uniform (nan for gibbs)                   sp_utils.py:30-31
    u[c, t]       update flag (1 True, 0 None)                        sp_utils.py:34-37
"""
import os
import sys
import json
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))), 'tests'))
import numpy as np
import scipy
import scipy.stats
import scipy.special

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   'tests', 'golden')


def _pb():
  import probayes as pb
  import probayes.prob as P
  # scipy>=1.15 frozen mvn lacks .fit while the class has it (prob.py:212-216):
  # run-time workaround only, the reference is not edited.
  P.SCIPY_DIST_METHODS = [m for m in P.SCIPY_DIST_METHODS if m != 'fit']
  return pb


from mcmc_examples import WORKLOADS, TFUN_WORKLOADS, DELTA_WORKLOADS, \
    SEGMENTED  # noqa: E402
# builders shared with tests
WORKLOADS = dict(WORKLOADS, **TFUN_WORKLOADS, **DELTA_WORKLOADS)


def _nan(v):
  return np.nan if v is None else float(v)


def run(name):
  """One workload; a SEGMENTED name runs its base workload's consecutive
  samplers (same process, same init, NumPy's global stream continuing)."""
  pb = _pb()
  segments = None
  if name in SEGMENTED:
    base, segments, n_chains = SEGMENTED[name]
    builder, params, _, _, seed0 = WORKLOADS[base]
    n_steps = int(sum(segments))
  else:
    builder, params, n_chains, n_steps, seed0 = WORKLOADS[name]
  keys = None
  arrs = {k: [] for k in ['v_x', 'v_p', 'p_x', 'p_p', 's', 't', 'u']}
  for c in range(n_chains):
    process, init, extra, kwds, keys = builder(pb, params)
    np.random.seed(seed0 + c)
    args = (init,) if extra is None else (init, extra)
    samples = []
    for stop in (segments or (n_steps,)):
      sampler = process.sampler(*args, stop=stop, **kwds)
      samples += list(process.walk(sampler))
    assert len(samples) == n_steps
    arrs['v_x'].append([[float(s.v[k]) for k in keys] for s in samples])
    arrs['v_p'].append([float(s.v.prob) for s in samples])
    arrs['p_x'].append([[float(s.p[k]) for k in keys] for s in samples])
    arrs['p_p'].append([float(s.p.prob) for s in samples])
    arrs['s'].append([_nan(s.s) for s in samples])
    arrs['t'].append([_nan(s.t) for s in samples])
    arrs['u'].append([1 if s.u else 0 for s in samples])
    # The summary path (sp.py:131-198) must agree with the per-step fields.
    summary = process(samples if segments is None else samples[-segments[-1]:])
    if segments is None:
      assert np.array_equal(np.ravel(summary.v[keys[0]]),
                          np.array(arrs['v_x'][-1])[:, 0])
      assert summary.u.count(True) == sum(arrs['u'][-1])
  out = {k: np.array(v, dtype=np.uint8 if k == 'u' else np.float64)
         for k, v in arrs.items()}
  if segments is not None:
    out['segments'] = np.array(segments, np.int64)
  out['seeds'] = np.arange(seed0, seed0 + n_chains, dtype=np.int64)
  out['keys'] = np.array(keys)
  for k, v in params.items():
    out['param_' + k] = np.asarray(v)
  meta = {'name': name, 'n_chains': n_chains, 'n_steps': n_steps,
          'seed0': seed0, 'numpy': np.__version__, 'scipy': scipy.__version__,
          'reference': 'probayes 0.0.8 (/root/reference)',
          'generator': 'tools/gen_golden.py'}
  out['meta'] = np.array(json.dumps(meta))
  os.makedirs(OUT, exist_ok=True)
  np.savez_compressed(os.path.join(OUT, name + '.npz'), **out)
  return out


if __name__ == '__main__':
  names = sys.argv[1:] or list(WORKLOADS) + list(SEGMENTED)
  for n in names:
    import time
    t0 = time.time()
    o = run(n)
    print('{:18s} chains={} steps={} accept={:.3f} {:.1f}s'.format(
        n, o['v_x'].shape[0], o['v_x'].shape[1], o['u'].mean(),
        time.time() - t0), flush=True)
