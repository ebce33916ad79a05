"""Nonce space sharded over GPUs, winner chosen by an all-reduce(min).

BASELINE config 4: one process per GPU.  Every search round is cut into
``world`` contiguous static shards; each rank mines its shard on its own GPU,
then ONE 24-byte all-reduce(MIN) of {counter found, go, ok} picks the winner
(the same counter a single GPU, or the CPU oracle, finds first in lowest
mode), spreads cancellation and reports a failed rank.  Inside a round the
ranks of one node also share a stop board, so the finder stops the other
GPUs' running kernels.  There is no data-path collective.

The search itself is implemented once, in C++ (``pow_group_*`` of
libpow_gpu.so, mpi_blockchain_amd/csrc/pow_group.cpp).  This module only
builds the group:

* :class:`RcclGroup` — the product path: RCCL (``ncclAllReduce``) called from
  C++, one process per GPU (bench.py at N > 1).
* :class:`ShardedMiner` — the same C++ rounds over torch.distributed's
  collectives (``pow_group_init_custom``): gloo on CPU, or several ranks that
  share one GPU (the multi-process GPU tests, bench.py's rehearsal), which
  RCCL refuses.

The reference has no mining-side collective (each MPI rank mines its own
template with its own rand() stream, node.cpp:302, 386); this is the
MI355X-native replacement for "all ranks search, first solution wins".
"""
from __future__ import annotations

import ctypes
import os
import uuid

from ._lib import (POW_REDUCE_MAX, POW_REDUCE_MIN, POW_REDUCE_SUM, REDUCE_FN, Block, GroupSearchInfo, check,
                   load)

_U64 = 1 << 64
_HALF = 1 << 63


def partition(start: int, count: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous static shard of [start, start+count) for `rank`
    (the Python mirror of pow_group_partition, tested equal)."""
    base, extra = divmod(count, world)
    lo = start + rank * base + min(rank, extra)
    return lo, base + (1 if rank < extra else 0)


def native_partition(start: int, count: int, rank: int, world: int) -> tuple[int, int]:
    """pow_group_partition of the C ABI (must equal :func:`partition`)."""
    s, n = ctypes.c_uint64(), ctypes.c_uint64()
    load().pow_group_partition(start, count, rank, world, ctypes.byref(s), ctypes.byref(n))
    return s.value, n.value


class _Group:
    """A ``pow_group``: the collective sharded search of include/pow_gpu.h."""

    miner = None
    L = None  # the library that made the group (the miner's)
    g = ctypes.c_void_p()

    def allreduce(self, vals, op: str = "min") -> list[int]:
        """In-place all-reduce of <= 8 uint64 over the group's ranks."""
        arr = (ctypes.c_uint64 * len(vals))(*vals)
        code = {"min": POW_REDUCE_MIN, "max": POW_REDUCE_MAX, "sum": POW_REDUCE_SUM}[op]
        check(self.L.pow_group_allreduce_u64(self.g, arr, len(vals), code), self.L)
        return list(arr)

    def mine(self, tmpl, start: int, count: int, difficulty: int, round_size: int = 0,
             epoch: int | None = None, any_solution: bool = False):
        """Lowest solving counter of [start, start+count) over all ranks
        (pow_group_mine), or with ``any_solution`` the first solution any GPU
        finds (pow_group_mine_any: the finder stops the node's other GPUs
        through the stop board).  Collective.  The same MineResult on every
        rank, or None (no solution / cancelled on some rank); raises PowError
        on every rank if any rank failed.  ``hashes`` and ``kernel_ms`` are
        this rank's, summed over the rounds."""
        from .miner import MineResult

        out = Block()
        ctr, hashes = ctypes.c_uint64(), ctypes.c_uint64()
        m = self.miner
        ep = m.epoch if epoch is None else epoch
        fn = m.L.pow_group_mine_any if any_solution else m.L.pow_group_mine
        rc = check(fn(self.g, ctypes.byref(tmpl), start, count, round_size, difficulty,
                      ctypes.byref(m._cancel), ep, ctypes.byref(out), ctypes.byref(ctr),
                      ctypes.byref(hashes)), self.L)
        if rc == 0:
            return None
        return MineResult(out, ctr.value, hashes.value, m.stats()["kernel_ms"])

    def info(self) -> dict:
        """The group as its transport sees it (pow_group_info): RCCL's
        ncclCommCount and ncclCommCuDevice for an RcclGroup; nranks and the
        miner's device for a custom group."""
        n, dev = ctypes.c_int(), ctypes.c_int()
        check(self.L.pow_group_info(self.g, ctypes.byref(n), ctypes.byref(dev)), self.L)
        return {"comm_count": n.value, "comm_device": dev.value}

    def last_search(self) -> dict:
        """This rank's part in the group's last :meth:`mine`
        (pow_group_last_search): whether the stop board was open and bound,
        the rounds, whether this rank's own launch found the solution, when
        that launch returned (CLOCK_MONOTONIC ns, = time.monotonic_ns()), and
        the wall ms in its launches and in the rounds' all-reduces."""
        i = GroupSearchInfo()
        check(self.L.pow_group_last_search(self.g, ctypes.byref(i)), self.L)
        return {k: getattr(i, k) for k, _ in GroupSearchInfo._fields_}

    def close(self) -> None:
        if self.g:
            self.L.pow_group_destroy(self.g)
            self.g = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class RcclGroup(_Group):
    """``pow_group_init``: the sharded search over RCCL (one 24-byte
    ``ncclAllReduce(ncclMin)`` per round, called from C++).  This is the form
    a C/C++ caller — the reference's node is C++ — uses; ranks exchange the
    128-byte RCCL id by any means (``from_torch`` uses torch.distributed)."""

    def __init__(self, miner, rank: int, world: int, unique_id: bytes, timeout_ms: int | None = None):
        """Joins the communicator; raises PowError (POW_ECOMM) if not every
        rank joined within `timeout_ms` (default: pow_group_init's 60 s)."""
        from ._lib import GROUP_ID_BYTES

        if len(unique_id) != GROUP_ID_BYTES:
            raise ValueError("unique_id must be 128 bytes")
        self.miner, self.rank, self.world = miner, rank, world
        self.L = miner.L
        self.g = ctypes.c_void_p()
        if timeout_ms is None:
            rc = miner.L.pow_group_init(miner.ctx, world, rank, unique_id, ctypes.byref(self.g))
        else:
            rc = miner.L.pow_group_init_within(miner.ctx, world, rank, unique_id, timeout_ms, ctypes.byref(self.g))
        check(rc, miner.L)

    @staticmethod
    def make_unique_id(L: ctypes.CDLL | None = None) -> bytes:
        """A fresh 128-byte id (ncclGetUniqueId) from library `L` (default:
        the shipped one; pass a miner's ``L`` to match its library)."""
        from ._lib import GROUP_ID_BYTES

        L = L or load()
        buf = ctypes.create_string_buffer(GROUP_ID_BYTES)
        check(L.pow_group_unique_id(buf), L)
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
                obj[0] = cls.make_unique_id(miner.L)
            except Exception as e:
                obj[0] = f"rank 0: {e}"
        dist.broadcast_object_list(obj, src=0, group=group)
        if isinstance(obj[0], str):
            raise RuntimeError(obj[0])
        return cls(miner, dist.get_rank(group), dist.get_world_size(group), obj[0])


def rccl_path(L: ctypes.CDLL | None = None) -> str:
    """The RCCL library file pow_group_* bind to (pow_group_rccl_path): the
    copy the process already loaded (torch's) if any."""
    L = L or load()
    buf = ctypes.create_string_buffer(4096)
    check(L.pow_group_rccl_path(buf, len(buf)), L)
    return buf.value.decode()


def loaded_rccl_files() -> list[str]:
    """Every librccl file mapped into this process (/proc/self/maps)."""
    out = []
    with open("/proc/self/maps") as f:
        for line in f:
            parts = line.split()
            if len(parts) >= 6 and os.path.basename(parts[-1]).startswith("librccl.so"):
                p = os.path.realpath(parts[-1])
                if p not in out:
                    out.append(p)
    return out


def torch_reduction(device=None, group=None):
    """f(vals, op) -> vals all-reduced over a torch.distributed group
    (op = POW_REDUCE_*).  uint64 words travel as int64: MIN/MAX shifted by
    2^63 (order-preserving), SUM as two's complement (mod 2^64)."""
    import torch
    import torch.distributed as dist

    ops = {POW_REDUCE_MIN: dist.ReduceOp.MIN, POW_REDUCE_MAX: dist.ReduceOp.MAX,
           POW_REDUCE_SUM: dist.ReduceOp.SUM}

    def f(vals: list[int], op: int) -> list[int]:
        if op == POW_REDUCE_SUM:
            enc = [v - _U64 if v >= _HALF else v for v in vals]
        else:
            enc = [v - _HALF for v in vals]
        t = torch.tensor(enc, dtype=torch.int64, device=device or "cpu")
        dist.all_reduce(t, op=ops[op], group=group)
        out = t.tolist()
        return [v % _U64 for v in out] if op == POW_REDUCE_SUM else [v + _HALF for v in out]

    return f


class ShardedMiner(_Group):
    """The sharded search (C++ rounds of pow_group_*) for one rank, with its
    all-reduce done by torch.distributed (``pow_group_init_custom``): gloo on
    CPU, or the ranks of a test that share one GPU.  With ``board`` (default)
    the ranks of one node share a stop board, its name made by rank 0 and
    broadcast.  ``miner=None`` builds a group that only carries
    :meth:`allreduce` (no GPU needed)."""

    def __init__(self, miner, rank: int, world: int, device=None, group=None, board: bool = True):
        import torch.distributed as dist

        self.miner, self.rank, self.world = miner, rank, world
        self.L = miner.L if miner is not None else load()
        self.g = ctypes.c_void_p()
        self.reduce_error: Exception | None = None
        red = torch_reduction(device, group)

        def cb(_user, vals, n, op):
            try:
                out = red([vals[i] for i in range(n)], op)
                for i, v in enumerate(out):
                    vals[i] = v
                return 0
            except Exception as e:  # reported through the C call's POW_ECOMM
                self.reduce_error = e
                return 1

        self._cb = REDUCE_FN(cb)  # kept alive as long as the group
        name = None
        if board and miner is not None and world <= 64:
            obj = [f"/pow_board_{os.getpid()}_{uuid.uuid4().hex[:12]}" if dist.get_rank(group) == 0 else None]
            dist.broadcast_object_list(obj, src=0, group=group)
            name = obj[0]
        check(self.L.pow_group_init_custom(miner.ctx if miner is not None else None, world, rank, self._cb, None,
                                           name.encode() if name else None, ctypes.byref(self.g)), self.L)
