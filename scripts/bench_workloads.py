#!/usr/bin/env python3
"""Secondary single-GPU measurements of the other BASELINE.json configs.

  cfg1  metrohast_norm1d (2 params, 60 iid obs in LDS, spherical delta,
        log ufun, joint prior), 128 chains -- and a 65 536-chain run
  cfg3  8-dim mvn CondCov Gibbs, 32 768 chains, 8 x 256 coordinate steps
  cfg5  3-component 2-D GMM, 32 768 chains (the per-GPU share of 262 144),
        2 000 steps, ESS/s (initial-positive-sequence ESS, min over dims,
        summed over chains, / kernel wall time)
One JSON line per workload.  Kernel time from the engine's HIP events.
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


def run(name, n, steps, rng='philox', spl=0, trace=True):
  spec = oracle.golden_spec(name)
  eng = Engine(spec)
  init = oracle.workloads.golden_init(name, n)
  eng.init_chains(init)
  eng.set_rng(rng, seed=11)
  eng.run(8)          # warm-up launch (code-object load stays untimed)
  if trace:
    eng.alloc_trace(steps, 1)
  eng.run(steps, steps_per_launch=spl)
  ms, launches = eng.last_run_ms()
  out = {'workload': name, 'chains': n, 'steps': steps,
         'chain_steps_per_s': n * steps / (ms / 1e3), 'kernel_ms': ms,
         'launches': launches, 'rng': rng}
  return eng, out


def main():
  import argparse
  ap = argparse.ArgumentParser()
  ap.add_argument('--only', default='cfg1,cfg3,cfg5',
                  help='comma-separated subset of cfg1,cfg3,cfg5')
  ap.add_argument('--no-trace', action='store_true',
                  help='cfg3 without the trace (arithmetic-only probe)')
  args = ap.parse_args()
  only = args.only.split(',')
  lines = []
  if 'cfg1' in only:
    eng, o = run('metrohast_norm1d', 128, 2000)
    eng.close()
    lines.append(dict(o, config='cfg1 (128 chains)'))
    eng, o = run('metrohast_norm1d', 65536, 1000)
    eng.close()
    lines.append(dict(o, config='cfg1 model at 65536 chains'))
  if 'cfg3' in only:
    eng, o = run('gibbs8', 32768, 8 * 256, trace=not args.no_trace)
    o['coordinate_steps_per_s'] = o.pop('chain_steps_per_s')
    o['hbm_gbs'] = o['coordinate_steps_per_s'] * (8 * 8 + 8 + 1 / 8) / 1e9
    eng.close()
    lines.append(dict(o, config='cfg3'))
  if 'cfg5' not in only:
    for line in lines:
      print(json.dumps(line), flush=True)
    return
  eng, o = run('gmm2', 32768, 2000)
  t0 = time.perf_counter()
  tr = eng.trace()
  eng.close()
  ess = [ess_ips(tr['v_x'][:, 500:, k]).sum() for k in range(2)]
  o['ess_min_dim'] = float(min(ess))
  o['ess_per_s'] = o['ess_min_dim'] / (o['kernel_ms'] / 1e3)
  o['ess_host_s'] = time.perf_counter() - t0
  lines.append(dict(o, config='cfg5 per-GPU share'))
  for line in lines:
    print(json.dumps(line), flush=True)


if __name__ == '__main__':
  main()
