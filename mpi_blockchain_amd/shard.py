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

import ctypes
from typing import Callable, Optional

NONE = (1 << 63) - 1  # "no solution" in the int64 all-reduce


def partition(start: int, count: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous static shard of [start, start+count) for `rank`."""
    base, extra = divmod(count, world)
    lo = start + rank * base + min(rank, extra)
    return lo, base + (1 if rank < extra else 0)


def round_plan(world: int, difficulty: int) -> tuple[int, int]:
    """First round size and cap of the adaptive plan (as pow_group_mine):
    ~4x the expected trials, at least 2^16 per rank; rounds then grow 4x up
    to 2^30 per rank."""
    big = world << 30
    return min(big, max(world << 16, 1 << (min(difficulty, 40) + 2))), big


def sharded_mine(search: Callable[[int, int], Optional[int]],
                 allreduce_min: Callable[[int], int],
                 start: int, count: int, round_size: int, rank: int, world: int,
                 difficulty: int = 0) -> Optional[int]:
    """Lowest solving counter of [start, start+count) over all ranks.

    search(s, n)        -> lowest solving counter in [s, s+n) on this rank, or None
    allreduce_min(v)    -> min of v over ranks (v = NONE when nothing found)
    round_size 0        -> adaptive rounds for `difficulty` (round_plan)
    Every rank returns the same value.
    """
    adaptive = round_size == 0
    if adaptive:
        round_size, big = round_plan(world, difficulty)
    done = 0
    while done < count:
        n = min(round_size, count - done)
        s, k = partition(start + done, n, rank, world)
        local = search(s, k) if k > 0 else None
        best = allreduce_min(NONE if local is None else local)
        if best != NONE:
            return best
        done += n
        if adaptive:
            round_size = min(big, round_size * 4)
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


class RcclGroup:
    """The same sharded search done natively: ``pow_group_*`` of
    libpow_gpu.so (mpi_blockchain_amd/csrc/pow_group.cpp) runs the rounds in
    C++ and calls RCCL itself (one 24-byte ``ncclAllReduce(ncclMin)`` per
    round for winner, cancellation and failure).  This is the form a C/C++
    caller — the reference's node is C++ — uses; ranks exchange the 128-byte
    RCCL id by any means (``from_torch`` uses torch.distributed)."""

    def __init__(self, miner, rank: int, world: int, unique_id: bytes):
        from ._lib import GROUP_ID_BYTES, check

        if len(unique_id) != GROUP_ID_BYTES:
            raise ValueError("unique_id must be 128 bytes")
        self.miner, self.rank, self.world = miner, rank, world
        self.g = ctypes.c_void_p()
        check(miner.L.pow_group_init(miner.ctx, world, rank, unique_id, ctypes.byref(self.g)))

    @staticmethod
    def make_unique_id() -> bytes:
        from ._lib import GROUP_ID_BYTES, check, load

        buf = ctypes.create_string_buffer(GROUP_ID_BYTES)
        check(load().pow_group_unique_id(buf))
        return buf.raw

    @classmethod
    def from_torch(cls, miner, group=None) -> "RcclGroup":
        """Collective over an initialised torch.distributed process group:
        rank 0 makes the id, every rank receives it, all join."""
        import torch.distributed as dist

        # Rank 0 always broadcasts (its error text if it could not make an id),
        # so no peer is left waiting in the broadcast or in ncclCommInitRank.
        obj = [None]
        if dist.get_rank(group) == 0:
            try:
                obj[0] = cls.make_unique_id()
            except Exception as e:
                obj[0] = f"rank 0: {e}"
        dist.broadcast_object_list(obj, src=0, group=group)
        if isinstance(obj[0], str):
            raise RuntimeError(obj[0])
        return cls(miner, dist.get_rank(group), dist.get_world_size(group), obj[0])

    def allreduce(self, vals, op: str = "min") -> list[int]:
        from ._lib import POW_REDUCE_MAX, POW_REDUCE_MIN, POW_REDUCE_SUM, check

        arr = (ctypes.c_uint64 * len(vals))(*vals)
        code = {"min": POW_REDUCE_MIN, "max": POW_REDUCE_MAX, "sum": POW_REDUCE_SUM}[op]
        check(self.miner.L.pow_group_allreduce_u64(self.g, arr, len(vals), code))
        return list(arr)

    def mine(self, tmpl, start: int, count: int, difficulty: int, round_size: int = 0,
             epoch: int | None = None, any_solution: bool = False):
        """Lowest solving counter of [start, start+count) over all ranks
        (pow_group_mine), or with ``any_solution`` the first solution any GPU
        finds (pow_group_mine_any: the finder stops the node's other GPUs
        through the stop board).  The same MineResult on every rank;
        ``hashes`` and ``kernel_ms`` are this rank's, summed over the rounds."""
        from ._lib import Block, check
        from .miner import MineResult

        out = Block()
        ctr, hashes = ctypes.c_uint64(), ctypes.c_uint64()
        m = self.miner
        ep = m.epoch if epoch is None else epoch
        fn = m.L.pow_group_mine_any if any_solution else m.L.pow_group_mine
        rc = check(fn(self.g, ctypes.byref(tmpl), start, count, round_size, difficulty,
                      ctypes.byref(m._cancel), ep, ctypes.byref(out), ctypes.byref(ctr),
                      ctypes.byref(hashes)))
        if rc == 0:
            return None
        return MineResult(out, ctr.value, hashes.value, m.stats()["kernel_ms"])

    def close(self) -> None:
        if self.g:
            self.miner.L.pow_group_destroy(self.g)
            self.g = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def native_partition(start: int, count: int, rank: int, world: int) -> tuple[int, int]:
    """pow_group_partition of the C ABI (must equal :func:`partition`)."""
    from ._lib import load

    s, n = ctypes.c_uint64(), ctypes.c_uint64()
    load().pow_group_partition(start, count, rank, world, ctypes.byref(s), ctypes.byref(n))
    return s.value, n.value


class ShardedMiner:
    """GPU-backed sharded search for one rank (one GPU per process) over
    torch.distributed.  With ``board=True`` the ranks of one node also share a
    stop board (its name broadcast from rank 0), so a rank's hit stops the
    others inside their running launches, as pow_group_* do natively."""

    def __init__(self, miner, rank: int, world: int, device=None, group=None, board: bool = False):
        self.miner, self.rank, self.world = miner, rank, world
        self.allreduce_min = torch_allreduce_min(device, group)
        self.board, self._searches = None, 0
        if board and world <= 64:
            import os
            import uuid

            import torch.distributed as dist

            from .miner import StopBoard

            obj = [f"/pow_board_{os.getpid()}_{uuid.uuid4().hex[:12]}" if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0, group=group)
            self.board = StopBoard(world, obj[0])
            dist.barrier(group=group)  # every rank has it mapped: the name can go
            self.board.unlink()

    def mine(self, tmpl, start: int, count: int, difficulty: int, round_size: int = 0,
             any_solution: bool = False):
        """Lowest solving counter over all ranks, or (``any_solution``) the
        lowest of the counters the ranks found first in the winning round."""
        if self.board is not None:
            self._searches += 1
            self.miner.bind_board(self.board, self.rank, 1 + (self._searches - 1) % 1023)

        def search(s, n):
            r = self.miner.mine(tmpl, s, n, difficulty, any_solution=any_solution)
            return None if r is None else r.counter

        try:
            return sharded_mine(search, self.allreduce_min, start, count,
                                (self.world << 32 if any_solution and not round_size else round_size),
                                self.rank, self.world, difficulty)
        finally:
            if self.board is not None:
                self.miner.bind_board(None)

    def close(self) -> None:
        if self.board is not None:
            self.miner.bind_board(None)
            self.board.close()
            self.board = None
