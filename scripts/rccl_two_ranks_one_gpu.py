"""The engine's RCCL collectives at world 2 on one card:
two processes, both on device 0, each an engine over its shard of the cfg5
model (dist.shard, global chain offsets); the ncclUniqueId travels over TCP
(dist.exchange_unique_id) and then

  * pbh_rccl_allreduce_max of (rank + 1) must give 2 on both ranks;
  * pbh_rccl_allgather_stats must hand both ranks every rank's per-chain
    statistics (sum, sumsq, n_acc, ESS), each block equal to that rank's own
    device reduction (trace_stats / trace_ess) bit for bit.

The parent never touches the GPU: it starts the ranks as child processes and
compares what they wrote.  One process per GPU is the production layout; two
ranks on one device would test the collectives' code path only -- and this
RCCL refuses it: ncclCommInitRank fails with "Duplicate GPU detected" on both
ranks (profiles/r05s2/rccl_one_card.txt), so world > 1 needs a real node.
usage: python scripts/rccl_two_ranks_one_gpu.py OUTDIR"""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

N_TOTAL, STEPS, WORLD, PORT = 8192, 64, 2, 29533


def rank_main(rank, outdir):
  import oracle
  from oracle.workloads import golden_init
  from probayes_amd import Engine
  from probayes_amd.dist import exchange_unique_id, shard
  off, n = shard(N_TOTAL, rank, WORLD)
  eng = Engine(oracle.golden_spec('gmm2'), device=0)
  eng.init_chains(_slice_init(golden_init('gmm2', N_TOTAL), off, n), chain_offset=off)
  eng.set_rng('philox', seed=7)
  eng.set_collect(moments=False)
  eng.alloc_trace(STEPS, 1)
  eng.run(STEPS)
  own = eng.trace_stats(0)
  own_ess = eng.trace_ess(STEPS // 4)
  uid = exchange_unique_id(rank, WORLD, Engine.rccl_unique_id() if rank == 0 else None,
                           port=PORT, timeout=60.0)
  eng.rccl_init(rank, WORLD, uid)
  mx = eng.rccl_allreduce_max(rank + 1.0)
  got = eng.rccl_allgather_stats()
  eng.close()
  np.savez(os.path.join(outdir, 'rank{}.npz'.format(rank)), off=off, n=n,
           sum=own['sum'], sumsq=own['sumsq'], n_acc=own['n_acc'], ess=np.asarray(own_ess),
           g_sum=got['sum'], g_sumsq=got['sumsq'], g_n_acc=got['n_acc'], g_ess=got['ess'],
           g_counts=got['counts'], mx=mx)


def _slice_init(init, off, n):
  """golden_init's chains [off, off + n) (a dict of per-variable arrays or
  one [N, d] array)."""
  if isinstance(init, dict):
    return {k: np.asarray(v)[off:off + n] for k, v in init.items()}
  return np.asarray(init)[off:off + n]


def main(outdir):
  os.makedirs(outdir, exist_ok=True)
  env = dict(os.environ, MASTER_ADDR='127.0.0.1')
  procs = [subprocess.Popen([sys.executable, '-u', os.path.abspath(__file__), outdir,
                             '--rank', str(r)], env=env,
                            stdout=open(os.path.join(outdir, 'rank{}.log'.format(r)), 'w'),
                            stderr=subprocess.STDOUT)
           for r in range(WORLD)]
  rcs = [p.wait(timeout=150) for p in procs]
  res = {'world': WORLD, 'chains': N_TOTAL, 'steps': STEPS, 'rank_rc': rcs}
  if any(rcs):
    print(json.dumps(res), flush=True)
    return 1
  r = [np.load(os.path.join(outdir, 'rank{}.npz'.format(k))) for k in range(WORLD)]
  ok = {'allreduce_max': all(float(x['mx']) == float(WORLD) for x in r),
        'counts': all(list(x['g_counts']) == [int(y['n']) for y in r] for x in r)}
  for key in ('sum', 'sumsq', 'n_acc', 'ess'):
    whole = np.concatenate([x[key] for x in r])
    ok[key] = all(np.array_equal(x['g_' + key], whole) for x in r)
  res.update(ok)
  print(json.dumps(res), flush=True)
  return 0 if all(ok.values()) else 1


if __name__ == '__main__':
  if '--rank' in sys.argv:
    rank_main(int(sys.argv[sys.argv.index('--rank') + 1]), sys.argv[1])
  else:
    sys.exit(main(sys.argv[1]))
