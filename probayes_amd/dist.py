"""Chain sharding across GPUs: one process per GPU.

Chains are independent, so the data path has no collective: rank r of W runs
the contiguous global chain ids [offset, offset + count) and keys its RNG by
global id (Philox) or by seeds[offset:offset + count] (legacy replay), which
makes every chain's trace identical for any W.  The single exchange is the
collection of per-chain moments: an RCCL all-gather over xGMI issued by the
engine (pbh_rccl_allgather_moments), or -- for CPU tests of this host logic
-- a torch.distributed gloo all-gather of the same [2d+1][count] block.
"""
import numpy as np


def shard(n_total, rank, world):
  """(offset, count) of rank's contiguous block; remainders go to low ranks."""
  if world < 1 or not 0 <= rank < world:
    raise ValueError('bad rank {} / world {}'.format(rank, world))
  base, rem = divmod(int(n_total), int(world))
  count = base + (1 if rank < rem else 0)
  offset = rank * base + min(rank, rem)
  return offset, count


def pack_moments(sum_, sumsq, n_acc):
  """[2d+1][N] block the engine's RCCL all-gather moves (pbhip.h)."""
  sum_, sumsq = np.asarray(sum_, np.float64), np.asarray(sumsq, np.float64)
  return np.concatenate([sum_.T, sumsq.T,
                         np.asarray(n_acc, np.float64)[None, :]], axis=0)


def unpack_gathered(blocks, d):
  """[W][2d+1][n] gathered blocks -> chain-major (sum [N, d], sumsq, n_acc)."""
  cat = np.concatenate(list(blocks), axis=1)
  return cat[:d].T, cat[d:2 * d].T, cat[2 * d].astype(np.int64)


class GlooCollective:
  """torch.distributed (gloo, CPU) stand-in for the engine's RCCL calls."""

  def __init__(self):
    import torch.distributed as dist
    self.dist = dist
    self.rank, self.world = dist.get_rank(), dist.get_world_size()

  def allgather_blocks(self, block):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(block))
    outs = [torch.empty_like(t) for _ in range(self.world)]
    self.dist.all_gather(outs, t)
    return np.stack([o.numpy() for o in outs])

  def allreduce_max(self, value):
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64)
    self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
    return float(t.item())
