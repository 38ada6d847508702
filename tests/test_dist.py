"""Multi-GPU host logic on CPU: world_size-2 gloo processes shard the chains
by global id, run their shard, and gather the per-chain moments; the result
must equal the unsharded run (SURVEY.md §8(e) invariance)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from probayes_amd.dist import shard, pack_moments, unpack_gathered

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shard_partition():
  for n in (1, 7, 64, 65536, 524288 + 3):
    for w in (1, 2, 3, 8):
      blocks = [shard(n, r, w) for r in range(w)]
      assert blocks[0][0] == 0
      for (o0, c0), (o1, _) in zip(blocks, blocks[1:]):
        assert o0 + c0 == o1
      assert sum(c for _, c in blocks) == n
      assert max(c for _, c in blocks) - min(c for _, c in blocks) <= 1
  with pytest.raises(ValueError):
    shard(10, 2, 2)


def test_pack_unpack_roundtrip():
  rs = np.random.RandomState(0)
  s, q, a = rs.normal(size=(5, 3)), rs.normal(size=(5, 3)), rs.randint(0, 9, 5)
  blk = pack_moments(s, q, a)
  s2, q2, a2 = unpack_gathered([blk[:, :2], blk[:, 2:]], 3)
  np.testing.assert_array_equal(s2, s)
  np.testing.assert_array_equal(q2, q)
  np.testing.assert_array_equal(a2, a)


WORKER = r'''
import os, sys, numpy as np
sys.path.insert(0, {root!r}); sys.path.insert(0, os.path.join({root!r}, 'tests'))
import torch.distributed as dist
dist.init_process_group('gloo')
import oracle
from probayes_amd.dist import shard, pack_moments, unpack_gathered, GlooCollective
rank, world = dist.get_rank(), dist.get_world_size()
spec = oracle.golden_spec('gmm2')
N, T = 37, 40
seeds = np.arange(1000, 1000 + N)
off, cnt = shard(N, rank, world)
out = oracle.run_mh(spec, np.zeros((cnt, 2)),
                    oracle.legacy_streams(spec, seeds[off:off + cnt], T))
x = out['v_x']
blk = pack_moments(x.sum(1), (x * x).sum(1), out['u'].sum(1))
col = GlooCollective()
# ragged shards: pad to the max count for the fixed-size all-gather
m = shard(N, 0, world)[1]
pad = np.zeros((blk.shape[0], m)); pad[:, :cnt] = blk
g = col.allgather_blocks(pad)
blocks = [g[r][:, :shard(N, r, world)[1]] for r in range(world)]
s, q, a = unpack_gathered(blocks, 2)
tmax = col.allreduce_max(float(rank))
if rank == 0:
  full = oracle.run_mh(spec, np.zeros((N, 2)), oracle.legacy_streams(spec, seeds, T))
  fx = full['v_x']
  assert np.array_equal(s, fx.sum(1)), 'sum'
  assert np.array_equal(q, (fx * fx).sum(1)), 'sumsq'
  assert np.array_equal(a, full['u'].sum(1)), 'n_acc'
  assert tmax == world - 1
  print('DIST_OK')
dist.destroy_process_group()
'''


def _free_port():
  s = socket.socket()
  s.bind(('127.0.0.1', 0))
  p = s.getsockname()[1]
  s.close()
  return p


def test_two_rank_gloo_sharded_run_matches_unsharded(tmp_path):
  script = tmp_path / 'worker.py'
  script.write_text(WORKER.format(root=ROOT))
  port = _free_port()
  procs = []
  for r in range(2):
    env = dict(os.environ, RANK=str(r), WORLD_SIZE='2', LOCAL_RANK=str(r),
               MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    procs.append(subprocess.Popen([sys.executable, str(script)], env=env,
                                  stdout=subprocess.PIPE,
                                  stderr=subprocess.STDOUT, text=True))
  outs = [p.communicate(timeout=240)[0] for p in procs]
  assert all(p.returncode == 0 for p in procs), outs
  assert 'DIST_OK' in outs[0], outs
