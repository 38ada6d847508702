"""Chain sharding across GPUs: one process per GPU.

Chains are independent, so the data path has no collective: rank r of W runs
the contiguous global chain ids [offset, offset + count) and keys its RNG by
global id (Philox) or by seeds[offset:offset + count] (legacy replay), which
makes every chain's trace identical for any W.  The single exchange is the
collection of per-chain statistics: ONE RCCL all-gather over xGMI issued by
the engine (pbh_rccl_allgather_stats: sum, sumsq, n_acc, ESS per chain,
ragged shards padded to the largest).

Control plane, standard library only (no torch): rank 0 hands its 128-byte
ncclUniqueId to the other ranks over TCP (exchange_unique_id).  TcpCollective
is the same star exchange carrying NumPy blocks; it stands in for the
engine's RCCL calls in CPU tests of the rank logic (tests/test_dist.py) and
packs blocks exactly like the engine (pack_stats / engine.unpack_stats).
"""
import io
import os
import socket
import struct
import time

import numpy as np


def shard(n_total, rank, world):
  """(offset, count) of rank's contiguous block; remainders go to low ranks."""
  if world < 1 or not 0 <= rank < world:
    raise ValueError('bad rank {} / world {}'.format(rank, world))
  base, rem = divmod(int(n_total), int(world))
  count = base + (1 if rank < rem else 0)
  offset = rank * base + min(rank, rem)
  return offset, count


def pack_stats(sum_, sumsq, n_acc, ess=None, n_max=None):
  """The [3d+1][n_max] block pbh_rccl_allgather_stats moves for one rank:
  rows sum[d], sumsq[d], n_acc, ess[d] (NaN when absent), zero padding past
  the rank's own count."""
  sum_, sumsq = np.asarray(sum_, np.float64), np.asarray(sumsq, np.float64)
  n, d = sum_.shape
  n_max = n if n_max is None else int(n_max)
  ess = np.full((n, d), np.nan) if ess is None else np.asarray(ess, np.float64)
  blk = np.zeros((3 * d + 1, n_max))
  blk[:, :n] = np.concatenate([sum_.T, sumsq.T,
                               np.asarray(n_acc, np.float64)[None, :], ess.T])
  return blk


# ---------------------------------------------------------------------------
# TCP control plane (stdlib)
# ---------------------------------------------------------------------------
def _send_msg(sock, payload):
  sock.sendall(struct.pack('<Q', len(payload)) + payload)


def _recv_exact(sock, n):
  buf = bytearray()
  while len(buf) < n:
    chunk = sock.recv(min(1 << 20, n - len(buf)))
    if not chunk:
      raise ConnectionError('peer closed the control connection')
    buf += chunk
  return bytes(buf)


def _recv_msg(sock):
  (n,) = struct.unpack('<Q', _recv_exact(sock, 8))
  return _recv_exact(sock, n)


def _connect(addr, port, timeout):
  t_end = time.monotonic() + timeout
  while True:
    try:
      return socket.create_connection((addr, port), timeout=timeout)
    except OSError:
      if time.monotonic() > t_end:
        raise
      time.sleep(0.05)


class CollectiveError(RuntimeError):
  """A rank failed inside a collective; every rank raises it."""


def fault_at(rank, step):
  """PBH_FAULT_GATHER='rank[:step]' (step 1 chains, 2 buffers, 3 packing;
  default 3): the engine's fault injection, read the same way here."""
  f = os.environ.get('PBH_FAULT_GATHER', '')
  if not f:
    return False
  r, _, st = f.partition(':')
  return int(r) == rank and int(st or 3) == step


def vote_message(what, status):
  """The error of a failed agreement (pbh_engine.hip vote_failure)."""
  if status >= 1:
    return ('{}: rank {} could not take part (the highest failing rank; see its '
            'own error)'.format(what, int(status) - 1))
  return '{}: a rank could not take part (see its own error)'.format(what)


class TcpCollective:
  """Star-topology exchange over TCP: rank 0 listens on (addr, port), the
  other ranks connect and announce their rank.  Used for the ncclUniqueId
  hand-off and, in CPU tests, in place of the engine's RCCL collectives."""

  def __init__(self, rank, world, addr='127.0.0.1', port=29511, timeout=120.0):
    self.rank, self.world = int(rank), int(world)
    self.peers = {}
    self.sock = None
    if self.world == 1:
      return
    if self.rank == 0:
      srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
      srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
      srv.bind((addr, port))
      srv.listen(self.world)
      srv.settimeout(timeout)
      try:
        while len(self.peers) < self.world - 1:
          conn, _ = srv.accept()
          conn.settimeout(timeout)
          (r,) = struct.unpack('<i', _recv_exact(conn, 4))
          if not 1 <= r < self.world or r in self.peers:
            # a stale process on the port, or a misconfigured launch: fail
            # now rather than time out or lose a rank's contribution
            conn.close()
            for c in self.peers.values():
              c.close()
            raise ConnectionError(
                'rank 0 got a connection announcing rank {} ({}; world {}, '
                'ranks connected: {})'.format(
                    r, 'already connected' if r in self.peers else 'out of range',
                    self.world, sorted(self.peers)))
          self.peers[r] = conn
      finally:
        srv.close()
    else:
      self.sock = _connect(addr, port, timeout)
      self.sock.sendall(struct.pack('<i', self.rank))

  def bcast_bytes(self, payload):
    """rank 0's payload on every rank."""
    if self.world == 1:
      return payload
    if self.rank == 0:
      for conn in self.peers.values():
        _send_msg(conn, payload)
      return payload
    return _recv_msg(self.sock)

  def allgather(self, arr):
    """[world, ...] stack of every rank's equally shaped array."""
    if self.world == 1:
      return np.asarray(arr)[None]
    buf = io.BytesIO()
    np.save(buf, np.ascontiguousarray(arr), allow_pickle=False)
    if self.rank == 0:
      parts = {0: buf.getvalue()}
      for r, conn in self.peers.items():
        parts[r] = _recv_msg(conn)
      blob = b''.join(struct.pack('<Q', len(parts[r])) + parts[r]
                      for r in range(self.world))
      for conn in self.peers.values():
        _send_msg(conn, blob)
    else:
      _send_msg(self.sock, buf.getvalue())
      blob = _recv_msg(self.sock)
    out, pos = [], 0
    for _ in range(self.world):
      (n,) = struct.unpack('<Q', blob[pos:pos + 8])
      out.append(np.load(io.BytesIO(blob[pos + 8:pos + 8 + n]),
                         allow_pickle=False))
      pos += 8 + n
    return np.stack(out)

  @staticmethod
  def _max(votes):
    """Elementwise max over ranks with NaN-DROPPING semantics (np.fmax): the
    operand-order-dependent behaviour a float max may have inside RCCL.  The
    votes are finite by construction, so the result does not depend on it."""
    return np.fmax.reduce(np.asarray(votes, np.float64), axis=0)

  def allreduce_max(self, value, ok=True):
    """pbh_rccl_allreduce_max: (value, status) under one max; a positive
    status (rank + 1 of a failed rank) makes every rank raise."""
    v = self._max(self.allgather(np.array([float(value),
                                           0. if ok else self.rank + 1.])))
    if v[1] != 0:
      raise CollectiveError(vote_message('allreduce_max', v[1]))
    return float(v[0])

  def agree(self, ok, n, what):
    """pbh_engine's rccl_agree: every rank votes (status, n, -n) -- status 0
    = ok, rank + 1 = this rank failed locally -- combined by one elementwise
    max; any positive status makes every rank raise the same error.
    Returns the largest n (the gather's padded width)."""
    v = self._max(self.allgather(
        np.array([0. if ok else self.rank + 1., float(n), -float(n)])))
    if v[0] != 0:
      raise CollectiveError(vote_message(what, v[0]))
    return int(v[1])

  def allgather_stats(self, sum_, sumsq, n_acc, ess=None):
    """The engine's pbh_rccl_allgather_stats contract on the CPU: agree on
    the padded width, then the [world][3d+2][n_max] all-gather whose last row
    carries each rank's count (element 0), behind the same agreements
    (chains, buffers, packing; PBH_FAULT_GATHER injects a local failure) so
    that a failing rank makes every rank fail, none wait.  Returns the
    [world][3d+1][n_max] statistics block and the counts."""
    n = np.asarray(sum_).shape[0]
    n_max = self.agree(not fault_at(self.rank, 1), n, 'allgather_stats')
    self.agree(not fault_at(self.rank, 2), n, 'allgather_stats (buffers)')
    ok = not fault_at(self.rank, 3)
    try:
      blk = pack_stats(sum_, sumsq, n_acc, ess, n_max=n_max)
      cnt = np.zeros((1, n_max))
      cnt[0, 0] = n
      blk = np.concatenate([blk, cnt])
    except Exception:   # this rank's failure is its vote
      ok, blk = False, None
    self.agree(ok, n, 'allgather_stats (packing)')
    got = self.allgather(blk)
    return got[:, :-1], got[:, -1, 0].astype(np.int64)

  def close(self):
    for conn in self.peers.values():
      conn.close()
    if self.sock is not None:
      self.sock.close()
    self.peers, self.sock = {}, None


def exchange_unique_id(rank, world, uid=None, addr='127.0.0.1', port=29511,
                       timeout=120.0):
  """rank 0's ncclUniqueId (128 bytes) on every rank, over TCP."""
  col = TcpCollective(rank, world, addr, port, timeout)
  try:
    got = col.bcast_bytes(bytes(uid) if rank == 0 else b'')
  finally:
    col.close()
  if len(got) != 128:
    raise ValueError('ncclUniqueId must be 128 bytes, got {}'.format(len(got)))
  return got
