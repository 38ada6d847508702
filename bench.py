#!/usr/bin/env python3
"""Headline benchmark: MH chain-steps/s on the cfg2 workload (BASELINE.json).

Workload (BASELINE.json configs[1]): 10-dim diagonal
Gaussian target prod_i N(mu_i, sigma_i^2), mu = linspace(-1, 1, 10), sigma =
linspace(0.5, 2, 10); random-walk proposal N(0, 0.5^2 I) (callable Delta of
norm.rvs); symmetric tran, log pscale, hastings/metropolis acceptance; init 0;
65 536 chains per GPU; production Philox RNG; the FULL trace (state, log-prob,
accept bit) of every step written to HBM -- the reference's walk() returns
every step (sp.py:281-295).

A bench "step" = one MH chain-step of every chain on every GPU.  The timed
region is exactly --steps steps (fused --steps-per-launch per kernel launch),
bracketed by a barrier + device sync on both sides; the reported time is the
max over ranks.  value = chains_per_gpu * n_gpus * steps / time.

Multi-GPU (weak scaling): one process per GPU (torch.distributed.run), chains
sharded by global id with no collective in the data path; one RCCL
all-gather of the per-chain moments at collection (timed separately).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
  sys.path.insert(0, ROOT)

METRIC = ('MH chain-steps/sec (whole node), 10-dim model, 65 536 chains, '
          '1/2/4/8 GPU')
D = 10
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


RNG_DESC = {
    'philox': 'philox4x32-10; fp64 Box-Muller normals on 52-bit uniforms '
              '(table-driven log/sqrt/sincos, a few ulp from libm)',
    'philox_f64': 'philox4x32-10; libm fp64 Box-Muller normals, reference '
                  'arithmetic',
    'xoshiro': 'xoshiro128** per chain; fp64 Box-Muller normals as philox',
    'philox_fp32': 'philox4x32-10; fp32 hardware Box-Muller normals on 24-bit '
                   'uniforms (|z| <= 5.77) -- comparison only, not fp64',
}


def cfg2_spec():
  from probayes_amd.spec import make_spec
  return make_spec(
      D,
      target={'kind': 'diag_gauss', 'mu': np.linspace(-1., 1., D),
              'sigma': np.linspace(0.5, 2., D)},
      proposal={'kind': 'gauss', 'loc': 0., 'scale': 0.5},
      scores='hastings', pscale='log',
      tran={'kind': 'const', 'value': 1.0, 'sym': True})


def bytes_per_chain_step(d):
  """Algorithmic HBM bytes of one chain-step with the full trace: the state
  x[d] and log-prob (fp64) plus one accept bit (wavefront ballot word)."""
  return 8.0 * d + 8.0 + 1.0 / 8.0


def cpu_baseline(budget_s=12.0):
  """The oracle (NumPy restatement of the reference, bit-exact per chain)
  timed on this host, including its legacy-MT19937 stream generation, on a
  bounded sample of the cfg2 workload."""
  import oracle
  spec = cfg2_spec()
  n, t = 2048, 8
  done, t0 = 0, time.perf_counter()
  reps = 0
  while time.perf_counter() - t0 < budget_s:
    seeds = np.arange(reps * n, (reps + 1) * n)
    streams = oracle.legacy_streams(spec, seeds, t)
    oracle.run_mh(spec, np.zeros((n, D)), streams)
    done += n * t
    reps += 1
  el = time.perf_counter() - t0
  return {'value': done / el, 'unit': 'chain-steps/s', 'cores': 1,
          'kind': 'port',
          'sample': '{} chains x {} steps x {} reps of cfg2 through '
                    'oracle.run_mh incl. per-chain RandomState streams, one '
                    'process (the reference SP itself: 877 chain-steps/s on 1 '
                    'core, BASELINE.md)'.format(n, t, reps)}


def measured_traffic(chains, launch_steps, rng, trace):
  """HBM bytes per launch of this exact launch shape (chains, steps in the
  launch, RNG mode), from the newest profiles/r*_traffic.json (rocprofv3 PMC
  passes, scripts/profile.sh), or None when no profile matches."""
  import glob
  files = sorted(glob.glob(os.path.join(ROOT, 'profiles', 'r*_traffic.json')))
  if not trace:
    return None
  for path in reversed(files):   # newest profile of this kernel and shape
    with open(path) as f:
      t = json.load(f)
    if (t.get('kernel', '').startswith('mh_pair_kernel') and
        t.get('chains') == chains and t.get('rng', 'philox_fp32') == rng and
        t.get('steps_per_launch') == launch_steps):
      return t['bytes_per_launch']
  return None


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument('--gpus', type=int, default=1)
  ap.add_argument('--steps', type=int, default=1000)
  ap.add_argument('--warmup', type=int, default=250,
                  help='untimed steps; a multiple of --steps-per-launch keeps '
                  'every dispatch the same shape as the timed ones')
  ap.add_argument('--chains', type=int, default=65536, help='per GPU')
  ap.add_argument('--steps-per-launch', type=int, default=250)
  ap.add_argument('--no-trace', action='store_true')
  ap.add_argument('--rng', default='philox',
                  choices=['philox', 'philox_f64', 'xoshiro', 'philox_fp32'])
  ap.add_argument('--moments', action='store_true',
                  help='keep in-kernel running moments (off: the trace is '
                  'reduced on the device after the timed region)')
  ap.add_argument('--no-cpu-baseline', action='store_true')
  ap.add_argument('--traffic-bytes', type=float, default=None,
                  help='HBM bytes per launch from a rocprofv3 PMC pass')
  args = ap.parse_args()

  world = int(os.environ.get('WORLD_SIZE', '1'))
  rank = int(os.environ.get('RANK', '0'))
  local = int(os.environ.get('LOCAL_RANK', '0'))
  if world != args.gpus:
    raise SystemExit('--gpus {} but WORLD_SIZE {}'.format(args.gpus, world))

  from probayes_amd import Engine   # loads libpbhip.so before any torch
  spec = cfg2_spec()
  n = args.chains
  eng = Engine(spec, device=local)
  from probayes_amd.dist import shard
  offset, n = shard(n * world, rank, world)   # weak scaling: n chains / GPU
  eng.init_chains(np.zeros((n, D)), chain_offset=offset)
  eng.set_rng(args.rng, seed=20261015)
  eng.set_collect(moments=args.moments or args.no_trace)
  if not args.no_trace:
    eng.alloc_trace(args.warmup + args.steps, 1)

  dist = None
  if world > 1:
    import torch.distributed as dist   # control plane only (gloo, CPU)
    dist.init_process_group('gloo')
    uid = [Engine.rccl_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    eng.rccl_init(rank, world, uid[0])

  def barrier():
    eng.sync()
    if world > 1:
      eng.rccl_allreduce_max(0.0)

  spl = args.steps_per_launch
  if args.warmup:
    eng.run(args.warmup, steps_per_launch=spl)
  barrier()
  t0 = time.perf_counter()
  eng.run(args.steps, steps_per_launch=spl, sync=False)
  eng.sync()
  el = time.perf_counter() - t0
  kern_ms, launches = eng.last_run_ms()
  barrier()
  if world > 1:
    el = eng.rccl_allreduce_max(el)
    t1 = time.perf_counter()
    if not args.no_trace and not args.moments:
      eng.trace_stats(args.warmup, args.steps)   # device reduction of the trace
    eng.rccl_allgather_moments()
    collect_ms = (time.perf_counter() - t1) * 1e3
  else:
    collect_ms = None

  total = float(n) * world * args.steps
  value = total / el
  bpcs = 0.0 if args.no_trace else bytes_per_chain_step(D)
  chain_steps_per_launch = n * (args.steps / max(launches, 1))
  avg_launch_s = kern_ms / 1e3 / max(launches, 1)
  achieved = bpcs * chain_steps_per_launch / avg_launch_s / 1e9
  if rank == 0:
    line = {
        'metric': METRIC, 'value': value, 'unit': 'chain-steps/s',
        'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': el * 1e3 / args.steps, 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None,
        'dtype': 'f32 normals, f64 chain' if args.rng == 'philox_fp32' else 'f64',
        'data': 'synthetic',
        'config': {'workload': 'cfg2: 10-dim diagonal-Gaussian random-walk '
                               'MH, {} chains/GPU, full trace every step'
                               .format(n),
                   'chains_per_gpu': n, 'dim': D,
                   'rng': RNG_DESC[args.rng],
                   'trace': not args.no_trace, 'steps_per_launch': spl,
                   'parallelism': 'chain-sharded x{}'.format(world)},
        'roofline': {'bound': 'hbm', 'achieved': achieved,
                     'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': achieved / HBM_PEAK_GBS,
                     'traffic': args.traffic_bytes if args.traffic_bytes
                                else measured_traffic(
                                    n, min(spl, args.steps), args.rng,
                                    not args.no_trace),
                     'bytes_per_chain_step': bpcs,
                     'kernel': ('mh_pair_kernel<10, {}>' if not os.environ.get('PBH_NO_PAIR') else 'mh_kernel<10, {}, DIAG, GAUSS>').format(args.rng.upper()),
                     'avg_launch_ms': avg_launch_s * 1e3,
                     'launches': launches},
        'kernel_chain_steps_per_s': n * args.steps / (kern_ms / 1e3),
    }
    if collect_ms is not None:
      line['rccl_allgather_ms'] = collect_ms
    if world == 1 and not args.no_cpu_baseline:
      line['cpu_baseline'] = cpu_baseline()
    print(json.dumps(line), flush=True)
  eng.close()
  if dist is not None:
    dist.destroy_process_group()


if __name__ == '__main__':
  main()
