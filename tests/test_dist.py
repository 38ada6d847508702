"""Multi-GPU host logic on CPU: world-2 processes run
bench.py's own rank logic (bench.run_rank: shard -> run -> device trace
statistics -> the one all-gather -> max-over-ranks time) with a CPU stand-in
for the engine (the oracle, bit-exact per chain, keyed by global chain id)
and the stdlib TCP collective in place of RCCL; the gathered statistics must
equal those of the unsharded run.  Also: the ncclUniqueId hand-off and the
ragged gather contract of pbh_rccl_allgather_stats (pad to the largest
shard, counts alongside)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from probayes_amd.dist import shard, pack_stats, TcpCollective
from probayes_amd.engine import unpack_stats

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


def test_pack_unpack_ragged_roundtrip():
  """pbh_rccl_allgather_stats' block layout: [world][3d+1][n_max] with zero
  padding past each rank's count; unpack_stats drops the padding and
  concatenates ranks in global chain order."""
  rs = np.random.RandomState(0)
  d, counts = 3, np.array([5, 4, 4])
  full = {'sum': rs.normal(size=(13, d)), 'sumsq': rs.normal(size=(13, d)),
          'n_acc': rs.randint(0, 9, 13), 'ess': rs.uniform(1, 9, (13, d))}
  blocks, o = [], 0
  for c in counts:
    sl = slice(o, o + c)
    blocks.append(pack_stats(full['sum'][sl], full['sumsq'][sl],
                             full['n_acc'][sl], full['ess'][sl], n_max=5))
    o += c
  got = unpack_stats(np.stack(blocks), counts, d)
  for k in ('sum', 'sumsq', 'n_acc', 'ess'):
    np.testing.assert_array_equal(got[k], full[k])
  assert np.isnan(pack_stats(full['sum'], full['sumsq'], full['n_acc'])[2 * d + 1:]).all()


ENGINE_STANDIN = r'''
import os, sys, time, numpy as np
sys.path.insert(0, {root!r})
import oracle

class OracleEngine:
  """CPU stand-in with the Engine methods bench.run_rank calls: every chain
  is the reference's (oracle.run_mh over per-chain legacy streams seeded by
  its GLOBAL id), so a rank's block equals the same block of an unsharded
  run."""
  def __init__(self, spec):
    self.spec = spec
  def init_chains(self, x0, chain_offset=0):
    self.x0, self.off = np.asarray(x0, float), int(chain_offset)
  def set_rng(self, rng, seed=0):
    self.seed = int(seed)
  def set_collect(self, moments=True):
    self.moments = moments
  def alloc_trace(self, cap, thin=1):
    self.cap, self.done = cap, 0
  def run(self, n, steps_per_launch=0, sync=True):
    self.done += n
  def sync(self):
    pass
  def last_run_ms(self):
    return 1.0, 1
  def trace_stats(self, first, count):
    n = len(self.x0)
    seeds = self.seed + self.off + np.arange(n)
    out = oracle.run_mh(self.spec, self.x0,
                        oracle.legacy_streams(self.spec, seeds, self.done))
    x = out['v_x'][:, first:first + count]
    self.stats = (x.sum(1), (x * x).sum(1), out['u'][:, first:first + count].sum(1))
    return self.stats
'''

WORKER = ENGINE_STANDIN + r'''
sys.path.insert(0, os.path.join({root!r}, 'tests'))
import bench
from probayes_amd.dist import TcpCollective
from probayes_amd.engine import unpack_stats
rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
col = TcpCollective(rank, world, '127.0.0.1', int(os.environ['MASTER_PORT']))

class Col:
  """TcpCollective with the EngineCollective interface of bench.py"""
  def allreduce_max(self, v):
    return col.allreduce_max(v)
  def gather_stats(self):
    s, q, a = eng.stats
    blk, counts = col.allgather_stats(s, q, a)
    return unpack_stats(blk, counts, bench.D)

eng = OracleEngine(bench.cfg2_spec())
res = bench.run_rank(eng, Col(), rank, world, chains_per_gpu=6, steps=12,
                     warmup=5, spl=4, rng='philox', seed=300)
st = res['stats']
if rank == 0:
  ref = OracleEngine(bench.cfg2_spec())
  ref.init_chains(np.zeros((6 * world, bench.D)), 0)
  ref.set_rng('philox', 300)
  ref.alloc_trace(17)
  ref.run(17)
  s, q, a = ref.trace_stats(5, 12)
  assert np.array_equal(st['sum'], s), 'sum'
  assert np.array_equal(st['sumsq'], q), 'sumsq'
  assert np.array_equal(st['n_acc'], a), 'n_acc'
  assert list(st['counts']) == [6] * world
  assert res['el'] >= 0 and res['offset'] == 0
  print('DIST_OK')
col.close()
'''


def _free_port():
  s = socket.socket()
  s.bind(('127.0.0.1', 0))
  p = s.getsockname()[1]
  s.close()
  return p


def _spawn(script, world, port):
  procs = []
  for r in range(world):
    env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world),
               LOCAL_RANK=str(r), MASTER_ADDR='127.0.0.1',
               MASTER_PORT=str(port))
    procs.append(subprocess.Popen([sys.executable, str(script)], env=env,
                                  stdout=subprocess.PIPE,
                                  stderr=subprocess.STDOUT, text=True))
  outs = [p.communicate(timeout=240)[0] for p in procs]
  assert all(p.returncode == 0 for p in procs), outs
  return outs


def test_two_rank_bench_rank_logic_matches_unsharded(tmp_path):
  script = tmp_path / 'worker.py'
  script.write_text(WORKER.format(root=ROOT))
  outs = _spawn(script, 2, _free_port())
  assert 'DIST_OK' in outs[0], outs


UID_WORKER = r'''
import os, sys
sys.path.insert(0, {root!r})
from probayes_amd.dist import exchange_unique_id, TcpCollective
rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
port = int(os.environ['MASTER_PORT'])
uid = bytes(range(128)) if rank == 0 else None
got = exchange_unique_id(rank, world, uid, '127.0.0.1', port)
assert got == bytes(range(128))
# ragged all-gather of statistics (counts 4, 3, 3 for 10 chains)
import numpy as np
from probayes_amd.dist import shard
off, n = shard(10, rank, world)
col = TcpCollective(rank, world, '127.0.0.1', port + 1)
s = np.arange(off, off + n, dtype=float)[:, None] * np.ones((1, 2))
blk, counts = col.allgather_stats(s, s * s, np.arange(off, off + n))
assert list(counts) == [shard(10, r, world)[1] for r in range(world)]
assert blk.shape == (world, 7, max(counts))
from probayes_amd.engine import unpack_stats
u = unpack_stats(blk, counts, 2)
assert np.array_equal(u['n_acc'], np.arange(10))
assert col.allreduce_max(rank) == world - 1
col.close()
print('UID_OK', rank)
'''


def test_unique_id_handoff_and_ragged_gather_three_ranks(tmp_path):
  script = tmp_path / 'uid.py'
  script.write_text(UID_WORKER.format(root=ROOT))
  outs = _spawn(script, 3, _free_port())
  assert all('UID_OK' in o for o in outs), outs


def test_rank0_rejects_a_duplicate_or_out_of_range_rank():
  """a stale process on the port announcing a rank already
  connected (or one outside 1..world-1) makes rank 0 fail at once."""
  import struct
  import threading
  from probayes_amd.dist import TcpCollective
  for bad in (1, 5):
    port = _free_port()
    err = []

    def rank0():
      try:
        TcpCollective(0, 3, '127.0.0.1', port, timeout=20)
      except ConnectionError as e:
        err.append(str(e))

    t = threading.Thread(target=rank0)
    t.start()
    socks = []
    for r in ((1, bad) if bad == 1 else (bad,)):
      for _ in range(200):
        try:
          s = socket.create_connection(('127.0.0.1', port), timeout=5)
          break
        except OSError:
          import time
          time.sleep(0.02)
      s.sendall(struct.pack('<i', r))
      socks.append(s)
    t.join(30)
    assert not t.is_alive()
    assert err and ('already connected' in err[0] or 'out of range' in err[0]), err
    for s in socks:
      s.close()


FAULT_WORKER = r'''
import os, sys
sys.path.insert(0, {root!r})
import numpy as np
from probayes_amd.dist import TcpCollective, CollectiveError, shard
rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
col = TcpCollective(rank, world, '127.0.0.1', int(os.environ['MASTER_PORT']), timeout=30)
off, n = shard(9, rank, world)
s = np.ones((n, 2))
try:
  col.allgather_stats(s, s, np.zeros(n))
  print('NO_ERROR', rank)
except CollectiveError as e:
  assert 'rank 1 could not take part' in str(e), str(e)
  # the protocol stays in step after a failure: the next collective works
  assert col.allreduce_max(rank) == world - 1
  print('FAILED_AS_ONE', rank)
col.close()
'''


@pytest.mark.parametrize('step', ['1', '2', '3'])
def test_a_rank_failing_inside_the_gather_fails_every_rank(tmp_path, monkeypatch, step):
  """Rank 1 fails locally at step `step` of the stats gather
  (PBH_FAULT_GATHER=1:step, the engine's fault injection): rank 0 fails with
  it instead of waiting in the all-gather, and both stay usable."""
  monkeypatch.setenv('PBH_FAULT_GATHER', '1:' + step)
  script = tmp_path / 'fault.py'
  script.write_text(FAULT_WORKER.format(root=ROOT))
  outs = _spawn(script, 2, _free_port())
  assert 'FAILED_AS_ONE 0' in outs[0] and 'FAILED_AS_ONE 1' in outs[1], outs


def test_failure_vote_survives_a_nan_dropping_max():
  """a NaN vote can vanish under a float max that drops
  NaN operands (fmax / compare-select, operand-order dependent); the vote is
  therefore a finite status (0 ok, rank + 1 failed), which every max keeps.
  The TCP stand-in reduces with np.fmax, the adversarial semantics."""
  from probayes_amd.dist import vote_message
  nan_votes = np.array([[0., 5., -5.], [np.nan, 4., -4.]])
  assert TcpCollective._max(nan_votes)[0] == 0.    # the old vote is lost
  for order in ([0, 1, 2], [2, 1, 0], [1, 0, 2]):
    votes = np.array([[0., 5., -5.], [2., 4., -4.], [0., 3., -3.]])[order]
    red = TcpCollective._max(votes)
    assert red[0] == 2. and red[1] == 5.
    assert 'rank 1 could not take part' in vote_message('x', red[0])
  # the engine's fallback fill (0x3F bytes) is a positive finite double
  fill = np.frombuffer(bytes([0x3F]) * 8, np.float64)[0]
  assert np.isfinite(fill) and 0. < fill < 1.
  assert 'a rank could not take part' in vote_message('x', fill)


MAIN_WORKER = ENGINE_STANDIN + r'''
import functools, io, json, contextlib
import bench
import probayes_amd
from probayes_amd.dist import TcpCollective
from probayes_amd.engine import unpack_stats
rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])


class MainEngine(OracleEngine):
  """The Engine interface bench.main() uses, RCCL calls included: the uid
  is 128 bytes as pbh_rccl_unique_id's, the collectives go over the stdlib
  TCP stand-in (its own port, next to the uid hand-off's)."""
  def __init__(self, spec, device=0):
    OracleEngine.__init__(self, spec)
    self.device = device
  @staticmethod
  def rccl_unique_id():
    return bytes(range(128))
  def rccl_init(self, rank_, world_, uid):
    assert uid == bytes(range(128)) and self.device == rank_
    self.col = TcpCollective(rank_, world_, '127.0.0.1',
                             int(os.environ['MASTER_PORT']) + 3)
  def rccl_allreduce_max(self, v):
    return self.col.allreduce_max(v)
  def rccl_allgather_stats(self):
    s, q, a = self.stats
    blk, counts = self.col.allgather_stats(s, q, a)
    return unpack_stats(blk, counts, bench.D)
  def seed_legacy(self, seeds):
    assert len(seeds) == len(self.x0) and seeds[0] == self.off
  def legacy_replay(self, k):
    assert k >= 1
  def reserve_replay(self, k):
    assert k >= 1
  def legacy_run(self, k, steps_per_launch=0, sync=True):
    assert k >= 1 and steps_per_launch >= 1
    self.run(k, steps_per_launch, sync)
  def server_info(self):
    # as if the timed run had been a resident-server command, so that main()
    # also times the launched form (PBH_SERVER=0) on a fresh engine
    return {{'active': False, 'commands': 1, 'launches': 1}}
  def stop_server(self):
    pass
  def close(self):
    if getattr(self, 'col', None) is not None:
      self.col.close()


probayes_amd.Engine = MainEngine        # main() imports it from the package
bench.lib_sha256 = lambda: 'standin'    # no library file needed on CPU
bench.cpu_baseline = functools.partial(bench.cpu_baseline, budget_s=0.3,
                                       chains=256)
sys.argv = ['bench.py', '--gpus', str(world), '--steps', '12', '--warmup',
            '5', '--chains', '6', '--steps-per-launch', '4']
buf = io.StringIO()
with contextlib.redirect_stdout(buf):
  bench.main()
out = buf.getvalue()
if rank == 0:
  lines = [l for l in out.splitlines() if l.strip()]
  assert len(lines) == 1, out
  line = json.loads(lines[0])
  assert line['n_gpus'] == world and line['steps'] == 12, line
  el = line['ms_per_step'] * 12 / 1e3            # the max over ranks
  assert abs(line['value'] * el / (6 * world * 12) - 1) < 1e-9, line
  assert line['cpu_baseline']['cores'] >= 1 and line['cpu_baseline']['value'] > 0
  assert line['rccl_allgather_ms'] >= 0
  assert line['roofline']['bound'] == 'hbm' and line['roofline']['frac'] > 0
  assert line['config']['parallelism'] == 'chain-sharded x{{}}'.format(world)
  assert line['scaling'] == 'weak'
  assert line['replay_chain_steps_per_s'] > 0 and 'REPLAY' in line['replay_config']
  assert line['launched_chain_steps_per_s'] > 0, line
  assert line['roofline']['kernel'].endswith('SRV>'), line['roofline']
  assert not line['launched']['kernel'].endswith('SRV>'), line['launched']
  print('MAIN_OK')
else:
  assert out == '', out
  print('QUIET_OK')
'''


def test_two_rank_bench_main_prints_one_scale_line(tmp_path):
  """bench.main() itself at world 2 -- the CPU baseline
  on rank 0 before the uid hand-off, the --gpus / WORLD_SIZE check, the
  RCCL barrier / max / all-gather calls (swapped for the TCP stand-in), the
  SCALE line's fields -- with exactly one line from rank 0 and nothing from
  the other rank, both exiting 0."""
  script = tmp_path / 'main.py'
  script.write_text(MAIN_WORKER.format(root=ROOT))
  outs = _spawn(script, 2, _free_port())
  assert 'MAIN_OK' in outs[0] and 'QUIET_OK' in outs[1], outs


def test_bench_main_rejects_a_world_size_mismatch(tmp_path):
  script = tmp_path / 'mismatch.py'
  script.write_text('import sys\nsys.path.insert(0, {root!r})\nimport bench\n'
                    'sys.argv = ["bench.py", "--gpus", "2"]\nbench.main()\n'
                    .format(root=ROOT))
  env = dict(os.environ, WORLD_SIZE='1', RANK='0', LOCAL_RANK='0')
  p = subprocess.run([sys.executable, str(script)], env=env, text=True,
                     stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                     timeout=120)
  assert p.returncode != 0 and 'WORLD_SIZE 1' in p.stdout, p.stdout
