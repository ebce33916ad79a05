"""Nonce space sharded over GPUs, winner chosen by an all-reduce(min).

BASELINE config 4: one process per GPU (``torch.distributed``, backend
``nccl`` = RCCL over xGMI on ROCm).  Every search round R counters wide is cut
into ``world`` contiguous static shards; each rank mines the LOWEST solving
counter of its shard on its own GPU (``pow_mine``), then one 8-byte
``all_reduce(MIN)`` picks the global winner — the same counter a single GPU (or
the CPU oracle) finds first, so the result is deterministic.  A non-empty
result ends the search on every rank (cancellation).  There is no data-path
collective: the only exchange is the 8-byte min per round.

The reference has no mining-side collective (each MPI rank mines its own
template with its own rand() stream, node.cpp:386); this is the MI355X-native
replacement for "all ranks search, first solution wins".
"""
from __future__ import annotations

from typing import Callable, Optional

NONE = (1 << 63) - 1  # "no solution" in the int64 all-reduce


def partition(start: int, count: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous static shard of [start, start+count) for `rank`."""
    base, extra = divmod(count, world)
    lo = start + rank * base + min(rank, extra)
    return lo, base + (1 if rank < extra else 0)


def sharded_mine(search: Callable[[int, int], Optional[int]],
                 allreduce_min: Callable[[int], int],
                 start: int, count: int, round_size: int, rank: int, world: int) -> Optional[int]:
    """Lowest solving counter of [start, start+count) over all ranks.

    search(s, n)        -> lowest solving counter in [s, s+n) on this rank, or None
    allreduce_min(v)    -> min of v over ranks (v = NONE when nothing found)
    Every rank returns the same value.
    """
    done = 0
    while done < count:
        n = min(round_size, count - done)
        s, k = partition(start + done, n, rank, world)
        local = search(s, k) if k > 0 else None
        best = allreduce_min(NONE if local is None else local)
        if best != NONE:
            return best
        done += n
    return None


def torch_allreduce_min(device=None, group=None) -> Callable[[int], int]:
    """8-byte all-reduce(MIN) through torch.distributed (RCCL when the
    process group is nccl and `device` is a GPU; gloo on CPU for tests)."""
    import torch
    import torch.distributed as dist

    buf = torch.zeros(1, dtype=torch.int64, device=device or "cpu")

    def f(v: int) -> int:
        buf.fill_(v)
        dist.all_reduce(buf, op=dist.ReduceOp.MIN, group=group)
        return int(buf.item())

    return f


class ShardedMiner:
    """GPU-backed sharded search for one rank (one GPU per process)."""

    def __init__(self, miner, rank: int, world: int, device=None, group=None):
        self.miner, self.rank, self.world = miner, rank, world
        self.allreduce_min = torch_allreduce_min(device, group)

    def mine(self, tmpl, start: int, count: int, difficulty: int, round_size: int = 1 << 31):
        def search(s, n):
            r = self.miner.mine(tmpl, s, n, difficulty)
            return None if r is None else r.counter

        return sharded_mine(search, self.allreduce_min, start, count, round_size, self.rank, self.world)
