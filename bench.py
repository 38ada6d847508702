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

Multi-GPU (weak scaling): one process per GPU (torch.distributed.run
launches them; nothing here imports torch), chains sharded by global id with
no collective in the data path; rank 0 hands its ncclUniqueId to the others
over TCP (stdlib), barriers and the max-over-ranks time are RCCL all-reduces,
and ONE RCCL all-gather collects the per-chain statistics (timed separately).
"""
import argparse
import json
import math
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


def _cpu_slice(args):
  """One process of the CPU baseline: cfg2 chain-steps of n chains through
  the vectorised NumPy restatement until the time budget is spent."""
  n, t, budget_s, seed = args
  from oracle.vector_mh import cfg2_run
  mu, sg = np.linspace(-1., 1., D), np.linspace(0.5, 2., D)
  done, t0 = 0, time.perf_counter()
  while True:
    cfg2_run(n, t, mu, sg, 0.5, seed + done)
    done += n * t
    el = time.perf_counter() - t0
    if el >= budget_s:
      return done, el


def _cpu_mask():
  """This process's CPU affinity as ranges ('0-255') and its count."""
  cpus = sorted(os.sched_getaffinity(0))
  rng, start = [], None
  for i, c in enumerate(cpus):
    if start is None:
      start = c
    if i + 1 == len(cpus) or cpus[i + 1] != c + 1:
      rng.append(str(start) if start == c else '{}-{}'.format(start, c))
      start = None
  return ','.join(rng), len(cpus)


def _cgroup_cpus():
  """The cgroup CPU quota in CPUs (cpu.max), or None when unlimited."""
  try:
    quota, period = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
    return None if quota == 'max' else float(quota) / float(period)
  except (OSError, ValueError):
    return None


def cpu_cores():
  """The CPUs this process may actually run on: the affinity mask, capped by
  the cgroup quota (a 16-CPU quota over a 256-CPU mask is 16 CPUs of time)."""
  mask, ncpu = _cpu_mask()
  quota = _cgroup_cpus()
  cores = ncpu if quota is None else max(1, min(ncpu, int(math.ceil(quota))))
  return cores, mask, ncpu, quota


def cpu_baseline(budget_s=6.0, chains=65536):
  """cfg2 on this host's cores, timed BEFORE the GPU is touched (the worker
  processes are forked from a process with no HIP state): the vectorised
  NumPy restatement (oracle/vector_mh.py, the reference's per-step arithmetic
  for all chains at once, every step recorded) at N = 65 536 on one core,
  then split over one process per usable CPU (cpu_cores: the affinity mask
  capped by the cgroup quota, so `cores` is what the processes really ran
  on).  The reference SP itself: 877 chain-steps/s on 1 core."""
  import multiprocessing as mp
  t = 16
  one_done, one_el = _cpu_slice((chains, t, budget_s, 1))
  cores, mask, ncpu, quota = cpu_cores()
  procs = min(cores, 1000)   # the box allows 1024 processes
  # independent chains per process; at least 4096 so that each process's
  # vectorised steps stay efficient when there are many
  per = max(-(-chains // procs), 4096)
  ctx = mp.get_context('fork')
  with ctx.Pool(procs) as pool:
    res = pool.map(_cpu_slice, [(per, t, budget_s, 100 + i) for i in range(procs)])
  rate_all = sum(d / e for d, e in res)
  return {'value': rate_all, 'unit': 'chain-steps/s', 'cores': procs,
          'kind': 'port',
          'single_core': one_done / one_el,
          'affinity': mask, 'affinity_cpus': ncpu, 'cgroup_cpu_quota': quota,
          'reference_sp_1core': 877.0,
          'sample': 'cfg2 (d = 10), oracle/vector_mh.py vectorised NumPy '
                    'restatement, every step recorded: {} chains x {}-step '
                    'runs for {:.0f} s on 1 core ({:.3g} chain-steps/s), then '
                    '{} processes (affinity mask {} = {} CPUs, cgroup quota {} '
                    'CPUs: {} usable) x {} chains for {:.0f} s each; the '
                    'reference SP: 877 chain-steps/s on 1 core '
                    '(BASELINE.md)'.format(chains, t, budget_s,
                                           one_done / one_el, procs, mask,
                                           ncpu,
                                           quota if quota else 'unlimited',
                                           cores, per, budget_s)}


def lib_sha256():
  """sha256 of the engine library this process loads (probayes_amd._lib)."""
  import hashlib
  from probayes_amd import _lib
  h = hashlib.sha256()
  with open(_lib.LIB_PATH, 'rb') as f:
    for blk in iter(lambda: f.read(1 << 20), b''):
      h.update(blk)
  return h.hexdigest()


def measured_traffic(chains, launch_steps, rng, trace, sha=None, srv=False):
  """HBM bytes per launch (per command when srv) of this exact shape (chains,
  steps in the launch or command, RNG mode, resident-server instance or
  launched) measured on THIS library build: the newest
  profiles/r*_traffic*.json (rocprofv3 FETCH_SIZE / WRITE_SIZE passes,
  scripts/profile_r06.sh + tools/collect_r06.py) whose lib_sha256 is the
  loaded library's and whose kernel instance is the one timed (`srv`: the
  server's one dispatch, its bytes divided over the steps commanded in its
  life); None when no profile of this binary and instance matches."""
  import glob
  if not trace:
    return None
  sha = sha or lib_sha256()
  files = sorted(glob.glob(os.path.join(ROOT, 'profiles', 'r*_traffic*.json')))
  for path in reversed(files):   # newest profile of this kernel and shape
    with open(path) as f:
      t = json.load(f)
    if (t.get('lib_sha256') == sha and
        t.get('kernel', '').startswith('mh_pair_kernel') and
        bool(t.get('srv', False)) == bool(srv) and
        t.get('chains') == chains and t.get('rng', 'philox_fp32') == rng and
        t.get('steps_per_launch') == launch_steps):
      return t['bytes_per_launch']
  return None


def kernel_label(args, n, srv=False):
  """The kernel the timed launches run (the engine's dispatch rules,
  pbh_kernels_impl.h launch_mh_pair_m / pair_full_form); srv: the timed run
  was a command to the resident server (its SRV instance)."""
  if os.environ.get('PBH_NO_PAIR'):
    return 'mh_kernel<10, {}, DIAG, GAUSS>'.format(args.rng.upper())
  mom = int(args.moments or args.no_trace)
  full = (args.rng == 'philox' and not mom and n % 32 == 0 and
          os.environ.get('PBH_PAIR_FULL', '1') != '0')
  return 'mh_pair_kernel<10, {}, MOM={}{}{}>'.format(
      args.rng.upper(), mom, ', FULL' if full else '', ', SRV' if srv else '')


class EngineCollective:
  """The engine's own RCCL collectives (pbh_rccl_*): the production path.
  host: a dist.TcpCollective for the barriers around the timed region (an
  RCCL call stops the resident server -- its kernel holds the device -- so
  the barrier before t0 is a host barrier; the max-over-ranks time and the
  statistics gather after it stay RCCL)."""

  def __init__(self, eng, host=None):
    self.eng = eng
    self.host = host

  def barrier(self):
    if self.host is not None:
      self.host.allreduce_max(0.0)
    else:
      self.eng.rccl_allreduce_max(0.0)

  def allreduce_max(self, v):
    return self.eng.rccl_allreduce_max(v)

  def gather_stats(self):
    return self.eng.rccl_allgather_stats()


def run_rank(eng, col, rank, world, chains_per_gpu, steps, warmup, spl, rng,
             trace=True, moments=False, seed=20261015, warmup_spl=None,
             gather=True):
  """One rank of the bench (weak scaling: chains_per_gpu chains per rank):
  shard the global chain ids, warm up, time exactly `steps` steps between
  barriers, take the max over ranks, then collect the per-chain statistics
  with the one all-gather.  eng: probayes_amd.Engine (or a CPU stand-in with
  the same methods, tests/test_dist.py); col: EngineCollective (RCCL) or
  dist.TcpCollective (world > 1), None for one rank."""
  from probayes_amd.dist import shard
  offset, n = shard(chains_per_gpu * world, rank, world)
  eng.init_chains(np.zeros((n, D)), chain_offset=offset)
  eng.set_rng(rng, seed=seed)
  eng.set_collect(moments=moments or not trace)
  if trace:
    eng.alloc_trace(warmup + steps, 1)

  def barrier():
    eng.sync()
    if col is not None:
      if hasattr(col, 'barrier'):
        col.barrier()
      else:
        col.allreduce_max(0.0)

  if warmup and warmup_spl is None and warmup <= 16:
    # a short warm-up runs as one-step runs, one pbh_run call each, so that
    # the host path the timed launch takes (ctypes -> pbh_run -> event
    # records -> launch) has run several times: the first timed enqueue is
    # 10-12 us after a single warm-up call, 7-8 us after this
    # (profiles/r03g_s20probe.jsonl)
    for _ in range(warmup):
      eng.run(1)
  elif warmup:
    eng.run(warmup, steps_per_launch=warmup_spl or spl)
  barrier()
  # the timed region: one library call (pbh_run_wait: the run and its wait)
  t0 = time.perf_counter()
  eng.run(steps, steps_per_launch=spl, sync=True)
  el = time.perf_counter() - t0
  kern_ms, launches = eng.last_run_ms()
  barrier()
  server = None
  if hasattr(eng, 'server_info'):
    server = eng.server_info()
    eng.stop_server()   # nothing else on this device waits behind it
  out = {'n': n, 'offset': offset, 'el': el, 'kern_ms': kern_ms,
         'launches': launches, 'server': server}
  if col is not None:
    out['el'] = col.allreduce_max(el)
    if not gather:
      return out
    t1 = time.perf_counter()
    if trace and not moments:
      eng.trace_stats(warmup, steps)   # device reduction of the timed steps
    out['stats'] = col.gather_stats()
    out['collect_ms'] = (time.perf_counter() - t1) * 1e3
  return out


def run_launched_rank(make_engine, col, rank, world, chains_per_gpu, steps,
                      warmup, spl, rng, trace, moments, warmup_spl):
  """The headline's shape with the resident server off (PBH_SERVER=0: every
  run launches the kernel, the engine's default for SP.sampler users), on a
  fresh engine, timed the same way (barrier + sync on both sides, max over
  ranks) after the headline: chain-steps/s of the whole job (not `value`)."""
  prev = os.environ.get('PBH_SERVER')
  os.environ['PBH_SERVER'] = '0'   # read at pbh_create
  try:
    eng = make_engine()
  finally:
    if prev is None:
      os.environ.pop('PBH_SERVER', None)
    else:
      os.environ['PBH_SERVER'] = prev
  try:
    res = run_rank(eng, col, rank, world, chains_per_gpu, steps, warmup, spl,
                   rng, trace=trace, moments=moments, warmup_spl=warmup_spl,
                   gather=False)
  finally:
    eng.close()
  kern_ms, launches = res['kern_ms'], res['launches']
  return {'chain_steps_per_s': float(chains_per_gpu) * world * steps / res['el'],
          'ms_per_step': res['el'] * 1e3 / steps,
          'events_us': kern_ms * 1e3, 'launches': launches,
          'host_us': (res['el'] - kern_ms / 1e3) * 1e6}


def run_replay_rank(make_engine, col, rank, world, chains_per_gpu, steps, warmup,
                    spl):
  """The parity-carrying mode on the same cfg2 shape:
  REPLAY -- the kernels read one NumPy RandomState(global chain id) stream
  per chain, generated on the device (pbh_legacy_seed; MT19937 + the polar
  legacy gauss, the reference's per-step draw order), and run the
  reference's arithmetic, so chains equal the reference CPU path's.  The
  draws go straight from the generator into the step (pbh_legacy_run: one
  fused kernel per launch; PBH_LEGACY_FUSED=0 runs stream generation + the
  REPLAY kernel instead).  Timed like the headline (barrier + sync on both
  sides, max over ranks): generation and the replay steps of exactly `steps`
  steps, the full trace written.  Returns chain-steps/s of the whole job (not
  `value`)."""
  from probayes_amd.dist import shard
  offset, n = shard(chains_per_gpu * world, rank, world)
  eng = make_engine()
  eng.init_chains(np.zeros((n, D)), chain_offset=offset)
  eng.set_rng('replay')
  eng.seed_legacy(offset + np.arange(n))
  eng.alloc_trace(warmup + steps, 1)
  chunk = max(1, min(spl, steps))
  if os.environ.get('PBH_LEGACY_FUSED', '1') == '0':
    # generation + REPLAY kernel: the stream buffer sized once for the
    # largest generation (a growth inside the timed region would be a
    # 100 MB-class hipMalloc there); the fused kernel (the default for this
    # form) writes no stream, so nothing is reserved for it
    eng.reserve_replay(max(chunk, min(spl, warmup) if warmup else 1))

  def advance(k):
    eng.legacy_run(k, steps_per_launch=chunk, sync=False)

  def barrier():
    eng.sync()
    if col is not None:
      if hasattr(col, 'barrier'):
        col.barrier()
      else:
        col.allreduce_max(0.0)

  if warmup:
    advance(warmup)
  barrier()
  t0 = time.perf_counter()
  advance(steps)
  eng.sync()
  el = time.perf_counter() - t0
  barrier()
  if col is not None:
    el = col.allreduce_max(el)
  eng.close()
  return float(chains_per_gpu) * world * steps / el, el


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
  ap.add_argument('--warmup-spl', type=int, default=None,
                  help='steps per warm-up launch (default: 1 for a warm-up '
                  'of <= 16 steps, else --steps-per-launch)')
  ap.add_argument('--traffic-bytes', type=float, default=None,
                  help='HBM bytes per launch from a rocprofv3 PMC pass')
  ap.add_argument('--no-replay', action='store_true',
                  help='skip the reference-identical REPLAY line fields')
  ap.add_argument('--no-launched', action='store_true',
                  help='skip the launched-form (PBH_SERVER=0) rate that is '
                  'reported beside a resident-server headline')
  args = ap.parse_args()

  world = int(os.environ.get('WORLD_SIZE', '1'))
  rank = int(os.environ.get('RANK', '0'))
  local = int(os.environ.get('LOCAL_RANK', '0'))
  if world != args.gpus:
    raise SystemExit('--gpus {} but WORLD_SIZE {}'.format(args.gpus, world))

  # the CPU baseline runs first on rank 0, before anything touches its GPU;
  # at world > 1 the other ranks wait for it at the ncclUniqueId hand-off
  # (exchange_unique_id), so every SCALE line carries the baseline too
  cpu = None
  if rank == 0 and not args.no_cpu_baseline:
    cpu = cpu_baseline()

  sha = lib_sha256()   # the binary the line (and its traffic profile) is of
  # this process is the host application and owns the device: spin-wait on
  # completion signals (hipDeviceScheduleSpin, process-wide, opt-in at
  # pbh_create; a short launch is seen to end ~2 us sooner)
  os.environ.setdefault('PBH_SPIN_FLAG', '1')
  # the resident sampling server (pbh_server_*): each timed run is a command
  # to a kernel launched during the warm-up (the steady-state lane-pair
  # kernel, chain state in registers); PBH_SERVER=0 launches per run
  os.environ.setdefault('PBH_SERVER', '1')
  from probayes_amd import Engine
  eng = Engine(cfg2_spec(), device=local)
  col = None
  if world > 1:
    # control plane: rank 0's ncclUniqueId over TCP (stdlib), then RCCL
    from probayes_amd.dist import exchange_unique_id
    addr = os.environ.get('MASTER_ADDR', '127.0.0.1')
    port = int(os.environ.get('MASTER_PORT', '29500')) + 1
    uid = exchange_unique_id(rank, world,
                             Engine.rccl_unique_id() if rank == 0 else None,
                             addr, port)
    eng.rccl_init(rank, world, uid)
    from probayes_amd.dist import TcpCollective
    col = EngineCollective(eng, TcpCollective(rank, world, addr, port + 1))
  spl = args.steps_per_launch
  res = run_rank(eng, col, rank, world, args.chains, args.steps, args.warmup,
                 spl, args.rng, trace=not args.no_trace, moments=args.moments,
                 warmup_spl=args.warmup_spl)
  n, el, kern_ms, launches = res['n'], res['el'], res['kern_ms'], res['launches']
  srv = bool(res.get('server') and res['server'].get('commands'))
  launched = None
  if srv and not args.no_launched:
    # the same shape launched per run (the engine's default form), after the
    # headline: reported beside value, never folded into it
    launched = run_launched_rank(lambda: Engine(cfg2_spec(), device=local), col,
                                 rank, world, args.chains, args.steps,
                                 args.warmup, spl, args.rng, not args.no_trace,
                                 args.moments, args.warmup_spl)
  replay = None
  if not args.no_replay:
    # after the headline's timed region and its collection, on a fresh engine
    replay = run_replay_rank(lambda: Engine(cfg2_spec(), device=local), col, rank,
                             world, args.chains, args.steps, args.warmup,
                             min(spl, 250))
  collect_ms = res.get('collect_ms')
  if 'stats' in res:   # every chain of every rank, once
    assert int(res['stats']['counts'].sum()) == args.chains * world

  total = float(args.chains) * world * args.steps
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
                                    not args.no_trace, sha, srv=srv),
                     'bytes_per_chain_step': bpcs,
                     'kernel': kernel_label(args, n, srv),
                     'avg_launch_ms': avg_launch_s * 1e3,
                     'launches': launches},
        'kernel_chain_steps_per_s': n * args.steps / (kern_ms / 1e3),
        # resident server: the timed run was a command to a kernel launched in
        # the warm-up; its kernel time is the command's device time (first
        # workgroup's sight of it to the last one's completion, s_memrealtime)
        'server': res.get('server'),
        'timing': ('device stamps of the resident server command'
                   if res.get('server') and res['server'].get('commands')
                   else 'HIP events around the launches'),
        # where the timed region's wall time went: the device time of the
        # launches / command (HIP events, or the server's stamps) and the
        # rest (host call, submission, completion signalling)
        'events_us': kern_ms * 1e3,
        'host_us': (el - kern_ms / 1e3) * 1e6,
        'lib_sha256': sha,
    }
    if collect_ms is not None:
      line['rccl_allgather_ms'] = collect_ms
    if launched is not None:
      # PBH_SERVER=0 on the same shape and clock: what SP.sampler users get
      line['launched_chain_steps_per_s'] = launched['chain_steps_per_s']
      line['launched'] = dict(launched, kernel=kernel_label(args, n, False),
                              note='PBH_SERVER=0, fresh engine, timed after '
                                   'the headline; not folded into value')
    if replay is not None:
      # the parity mode (reference-identical chains), same shape and clock;
      # reported beside value, never folded into it
      line['replay_chain_steps_per_s'] = replay[0]
      line['replay_ms_per_step'] = replay[1] * 1e3 / args.steps
      line['replay_config'] = ('REPLAY: per-chain NumPy RandomState(global '
                               'chain id) streams generated on the device '
                               '(MT19937 + polar legacy gauss) and the '
                               'reference arithmetic; generation inside the '
                               'timed region, fused into the step '
                               '(pbh_legacy_run)')
    if cpu is not None:
      line['cpu_baseline'] = cpu
    print(json.dumps(line), flush=True)
  if col is not None and getattr(col, 'host', None) is not None:
    col.host.close()
  eng.close()


if __name__ == '__main__':
  main()
