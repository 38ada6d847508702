#!/usr/bin/env python3
"""Secondary single-GPU measurements of the other BASELINE.json configs.

  cfg1  metrohast_norm1d (2 params, 60 iid obs in LDS, spherical delta,
        log ufun, joint prior), 128 chains -- and a 65 536-chain run
  cfg3  8-dim mvn CondCov Gibbs, 32 768 chains, 8 x 256 coordinate steps
  cfg5  3-component 2-D GMM, 32 768 chains (the per-GPU share of 262 144),
        2 000 steps, ESS/s (initial-positive-sequence ESS computed on the
        device from the resident trace, min over dims, summed over chains, /
        kernel time)
  lik   likelihoods.py bool_perm_freq: 2^28 rows x 2 columns (naive-Bayes
        table shape of examples/naive), HBM read stream
  legacy  cfg2 in the reference-identical REPLAY mode: the per-chain NumPy
        RandomState streams generated on the device, then the reference-
        arithmetic kernel over them (65 536 chains x 250 steps)
One JSON line per workload.  Kernel time from HIP events.  Each line carries
a roofline object (algorithmic HBM bytes / kernel time against 8 TB/s) and a
cpu_baseline: the oracle (the NumPy restatement of the reference, bit-exact
on the golden vectors) timed on a bounded sample on one host core.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))

import oracle  # noqa: E402  (specs of the golden workloads only)
from probayes_amd import Engine  # noqa: E402


def ess_ips(x):
  """Per-chain ESS of x [N, T] (Geyer initial positive sequence)."""
  n, t = x.shape
  xc = x - x.mean(axis=1, keepdims=True)
  f = np.fft.rfft(xc, n=2 * t, axis=1)
  ac = np.fft.irfft(f * np.conj(f), axis=1)[:, :t]
  ac /= np.maximum(ac[:, :1], 1e-300)
  m = (t - 1) // 2
  pairs = ac[:, 1:2 * m + 1:2] + ac[:, 2:2 * m + 2:2]      # rho_k + rho_k+1
  neg = pairs <= 0
  first = np.where(neg.any(axis=1), neg.argmax(axis=1), m)
  keep = np.arange(m)[None, :] < first[:, None]
  s = np.sum(np.where(keep, pairs, 0.), axis=1)
  return t / np.maximum(1.0 + 2.0 * s, 1e-12)


PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md)


def roofline(bytes_per_unit, units, ms, kernel):
  gbs = bytes_per_unit * units / (ms / 1e3) / 1e9
  return {'bound': 'hbm', 'achieved': gbs, 'peak': PEAK_GBS, 'unit': 'GB/s',
          'frac': gbs / PEAK_GBS, 'traffic': None,
          'bytes_per_unit': bytes_per_unit, 'kernel': kernel}


def cpu_chain_rate(name, n, t, budget_s):
  """Oracle chain-steps (or coordinate steps) per second on one core,
  including its legacy-MT19937 stream generation."""
  spec = oracle.golden_spec(name)
  run_ = oracle.run_gibbs if spec['scores'] == 'gibbs' else oracle.run_mh
  done, reps, t0 = 0, 0, time.perf_counter()
  while time.perf_counter() - t0 < budget_s:
    seeds = np.arange(reps * n, (reps + 1) * n)
    run_(spec, oracle.workloads.golden_init(name, n),
         oracle.legacy_streams(spec, seeds, t))
    done += n * t
    reps += 1
  el = time.perf_counter() - t0
  return {'value': done / el, 'unit': 'chain-steps/s', 'cores': 1,
          'kind': 'port',
          'sample': '{} chains x {} steps x {} reps of {} through the oracle '
                    'incl. per-chain RandomState streams'.format(n, t, reps, name)}


def run(name, n, steps, rng='philox', spl=0, trace=True):
  spec = oracle.golden_spec(name)
  eng = Engine(spec)
  init = oracle.workloads.golden_init(name, n)
  eng.init_chains(init)
  eng.set_rng(rng, seed=11)
  eng.set_collect(moments=not trace)   # with a trace: device trace_stats
  eng.run(8)          # warm-up launch (code-object load stays untimed)
  if trace:
    eng.alloc_trace(steps, 1)
  eng.run(steps, steps_per_launch=spl)
  ms, launches = eng.last_run_ms()
  out = {'workload': name, 'chains': n, 'steps': steps,
         'chain_steps_per_s': n * steps / (ms / 1e3), 'kernel_ms': ms,
         'launches': launches, 'rng': rng}
  return eng, out


def bench_bool_perm_freq(cpu, budget_s):
  """likelihoods.py:45-101 at 2^28 rows x 2 columns, input resident in HBM;
  the kernel reads every byte once (cols bytes per row)."""
  from probayes_amd.likelihoods import bool_counts
  from oracle.likelihoods import bool_perm_counts
  rows, cols = 1 << 28, 2
  a = np.random.RandomState(3).randint(0, 2, size=(rows, cols),
                                       dtype=np.uint8).view(bool)
  counts, ms = bool_counts(a, reps=5)
  assert counts.sum() == rows
  o = {'workload': 'bool_perm_freq', 'rows': rows, 'cols': cols,
       'rows_per_s': rows / (ms / 1e3), 'kernel_ms': ms,
       'roofline': roofline(cols, rows, ms,
                           'bool_perm_direct<2> + bool_perm_reduce'),
       'config': 'likelihoods.py bool_perm_freq, naive-Bayes table shape'}
  if cpu:
    n = 1 << 22
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
      bool_perm_counts(a[:n])
      done += n
    el = time.perf_counter() - t0
    o['cpu_baseline'] = {'value': done / el, 'unit': 'rows/s', 'cores': 1,
                         'kind': 'port',
                         'sample': '{} rows x {} cols through '
                                   'oracle.bool_perm_counts (np.bincount); '
                                   'the reference loops over rows in '
                                   'Python'.format(n, cols)}
  return o


def bench_legacy_replay():
  """cfg2 reference-identical: device RandomState streams + REPLAY kernel."""
  spec = oracle.golden_spec('diag10')
  n, t = 65536, 250
  eng = Engine(spec)
  eng.init_chains(np.zeros((n, 10)))
  eng.set_rng('replay')
  eng.seed_legacy(np.arange(n))
  # warm-up (code objects load lazily; the first call of a size allocates
  # the 1.4 GB stream buffer, which later calls of that size reuse)
  eng.legacy_replay(t)
  eng.run(8)
  t0 = time.perf_counter()
  eng.legacy_replay(t)
  gen_s = time.perf_counter() - t0
  eng.alloc_trace(t, 1)
  eng.run(t)
  ms, launches = eng.last_run_ms()
  eng.close()
  return {'workload': 'diag10 replay (reference-identical)', 'chains': n,
          'steps': t, 'stream_gen_ms': gen_s * 1e3,
          'stream_draws_per_s': n * t * 11 / gen_s,
          'replay_kernel_ms': ms,
          'chain_steps_per_s_kernel': n * t / (ms / 1e3),
          'chain_steps_per_s_with_streams': n * t / (ms / 1e3 + gen_s),
          'config': 'cfg2 shape, REPLAY mode fed by pbh_legacy_replay'}


def bench_linreg(cpu, budget_s):
  """gibbs_linreg user-conditional Gibbs (60 observations), PHILOX:
  65 536 chains x 1 000 coordinate steps per launch, full trace on device."""
  from oracle.linreg import linreg_streams, run_linreg
  from probayes_amd import linreg
  rs = np.random.RandomState(321)
  x = rs.normal(0, 1, size=60)
  y = rs.normal(1.5 * x - 1., 0.5)
  n, t = 65536, 1000
  init = np.tile([-0.9, 1.4, 0.6], (n, 1))
  ms = linreg.run(x, y, init, t, rng='philox', seed=1, reps=5,
                  trace=False)['ms']
  o = {'workload': 'gibbs_linreg (60 obs) PHILOX', 'chains': n, 'steps': t,
       'kernel_ms': ms, 'coordinate_steps_per_s': n * t / (ms / 1e3),
       'roofline': roofline(4 * 8, n * t, ms, 'linreg_gibbs_kernel<false>'),
       'config': 'user-tfun Gibbs, examples/mcmc/gibbs_linreg.py model'}
  if cpu:
    m, tc = 1024, 30
    done, reps, t0 = 0, 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
      st = linreg_streams(np.arange(reps * m, (reps + 1) * m), tc, 60)
      run_linreg(x, y, init[:m], st)
      done += m * tc
      reps += 1
    el = time.perf_counter() - t0
    o['cpu_baseline'] = {
        'value': done / el, 'unit': 'coordinate-steps/s', 'cores': 1,
        'kind': 'port',
        'sample': '{} chains x {} steps x {} reps through oracle.run_linreg '
                  'incl. per-chain RandomState streams'.format(m, tc, reps)}
  return o


def main():
  import argparse
  ap = argparse.ArgumentParser()
  ap.add_argument('--only', default='cfg1,cfg3,cfg5,lik,legacy,linreg',
                  help='comma-separated subset of cfg1,cfg3,cfg5,lik,legacy,'
                       'linreg')
  ap.add_argument('--no-cpu-baseline', action='store_true')
  ap.add_argument('--cpu-budget', type=float, default=4.0,
                  help='seconds of oracle work per cpu_baseline')
  ap.add_argument('--no-trace', action='store_true',
                  help='cfg3 / cfg5 without the trace (arithmetic-only probe)')
  args = ap.parse_args()
  only = args.only.split(',')
  cpu = not args.no_cpu_baseline
  lines = []
  if 'cfg1' in only:
    eng, o = run('metrohast_norm1d', 128, 2000)
    eng.close()
    lines.append(dict(o, config='cfg1 (128 chains)'))
    eng, o = run('metrohast_norm1d', 65536, 1000)
    eng.close()
    o['roofline'] = roofline(2 * 8 + 8 + 1 / 8, 65536 * 1000, o['kernel_ms'],
                             'mh_kernel<2, PHILOX, NORM_IID, SPHERE>')
    if cpu:
      o['cpu_baseline'] = cpu_chain_rate('metrohast_norm1d', 256, 8,
                                         args.cpu_budget)
    lines.append(dict(o, config='cfg1 model at 65536 chains'))
  if 'cfg3' in only:
    eng, o = run('gibbs8', 32768, 8 * 256, trace=not args.no_trace)
    o['coordinate_steps_per_s'] = o.pop('chain_steps_per_s')
    o['hbm_gbs'] = o['coordinate_steps_per_s'] * (8 * 8 + 8 + 1 / 8) / 1e9
    eng.close()
    o['roofline'] = roofline(8 * 8 + 8 + 1 / 8, 32768 * 8 * 256,
                             o['kernel_ms'], 'gibbs_fast_kernel<8, 2>')
    if cpu:
      o['cpu_baseline'] = dict(cpu_chain_rate('gibbs8', 256, 16,
                                              args.cpu_budget),
                               unit='coordinate-steps/s')
    lines.append(dict(o, config='cfg3'))
  if 'lik' in only:
    lines.append(bench_bool_perm_freq(cpu, args.cpu_budget))
  if 'legacy' in only:
    lines.append(bench_legacy_replay())
  if 'linreg' in only:
    lines.append(bench_linreg(cpu, args.cpu_budget))
  if 'cfg5' not in only:
    for line in lines:
      print(json.dumps(line), flush=True)
    return
  eng, o = run('gmm2', 32768, 2000, trace=not args.no_trace)
  if args.no_trace:
    eng.close()
    lines.append(dict(o, config='cfg5 per-GPU share, no trace'))
    for line in lines:
      print(json.dumps(line), flush=True)
    return
  # ESS on the device from the resident trace (no host copy of it):
  # pbh_trace_ess, Geyer's initial positive sequence per chain and dim
  eng.trace_ess(500)   # warm-up (code-object load)
  eng.trace_ess_total(500)
  ts, tp = [], []
  for _ in range(5):   # the calls' medians
    t0 = time.perf_counter()
    tot = eng.trace_ess_total(500)     # the metric: per-dim sums on the device
    t1 = time.perf_counter()
    ess_dev = eng.trace_ess(500)       # per-chain values copied back
    tp.append(time.perf_counter() - t1)
    ts.append(t1 - t0)
  o['ess_device_s'] = float(np.median(ts))
  o['ess_device_s_calls'] = [round(t, 6) for t in ts]
  o['ess_per_chain_call_s'] = float(np.median(tp))
  eng.close()
  ess = ess_dev.sum(axis=0)
  assert np.allclose(tot, ess, rtol=1e-12), (tot, ess)
  o['ess_min_dim'] = float(tot.min())
  # ESS per second of sampling kernel time, and end to end: sampling plus the
  # device ESS of its trace (ESS divided by wall)
  o['ess_per_s'] = o['ess_min_dim'] / (o['kernel_ms'] / 1e3)
  o['ess_per_s_end_to_end'] = o['ess_min_dim'] / (o['kernel_ms'] / 1e3 +
                                                  o['ess_device_s'])
  o['roofline'] = roofline(2 * 8 + 8 + 1 / 8, 32768 * 2000, o['kernel_ms'],
                           'mh_gmm_quad_kernel<2, 3>' if os.environ.get('PBH_GMM_LANES', '4') != '2' else 'mh_gmm_lanes_kernel<2, 3, 2>')
  if cpu:
    o['cpu_baseline'] = cpu_chain_rate('gmm2', 512, 8, args.cpu_budget)
  lines.append(dict(o, config='cfg5 per-GPU share'))
  for line in lines:
    print(json.dumps(line), flush=True)


if __name__ == '__main__':
  main()
