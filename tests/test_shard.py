"""Sharded search (pow_group_*, mpi_blockchain_amd/shard.py), CPU only.

The search rounds themselves run in C++ (csrc/pow_group.cpp) and need a GPU:
tests/test_shard_gpu.py drives them with 1, 2 and 4 ranks.  Here: the static
partition (Python mirror == C ABI), and the custom-reduction group
(pow_group_init_custom over torch.distributed gloo) at world size 2 and 4 in
real processes: its joining barrier, the uint64 encoding of min/max/sum, and
the checks a group without a GPU context makes."""
import os
import socket

import pytest

from mpi_blockchain_amd.shard import partition


def test_partition_covers_range():
    for count in (0, 1, 7, 62, 1000, 2**32 + 3):
        for world in (1, 2, 3, 4, 8):
            parts = [partition(100, count, r, world) for r in range(world)]
            assert parts[0][0] == 100
            for (s0, n0), (s1, _) in zip(parts, parts[1:]):
                assert s0 + n0 == s1
            assert sum(n for _, n in parts) == count


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


U64MAX = (1 << 64) - 1


def _custom_group_worker(rank, world, port, q):
    import ctypes

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mpi_blockchain_amd import _lib
    from mpi_blockchain_amd.shard import ShardedMiner

    out = {}
    with ShardedMiner(None, rank, world) as g:  # no GPU context: collectives only
        # the extremes of the uint64 range survive the int64 transport
        vals = [rank, U64MAX - rank, (1 << 63) + rank, 7 if rank == world - 1 else U64MAX]
        out["min"] = g.allreduce(vals, "min")
        out["max"] = g.allreduce(vals, "max")
        out["sum"] = g.allreduce([rank + 1, (1 << 63) + rank, U64MAX], "sum")
        # the round consensus word {counter, go, ok}: one rank cancelled
        out["consensus"] = g.allreduce([U64MAX if rank else 12345, 0 if rank == world - 1 else 1, 1], "min")
        blk = _lib.Block()
        out["info"] = g.info()
        out["mine_rc"] = _lib.load().pow_group_mine(g.g, ctypes.byref(blk), 0, 1, 0, 9, None, 0, ctypes.byref(blk),
                                                    None, None)
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_custom_group_collectives(world):
    """pow_group_init_custom over gloo in `world` processes: every rank joins
    (the init barrier checks the rank count), min/max/sum are exact over the
    whole uint64 range, and a group without a context refuses to mine."""
    import torch.multiprocessing as mp

    from mpi_blockchain_amd import _lib

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_custom_group_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        out = dict(q.get(timeout=120) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    want_min = [0, U64MAX - (world - 1), 1 << 63, 7]
    want_max = [world - 1, U64MAX, (1 << 63) + world - 1, U64MAX]
    want_sum = [world * (world + 1) // 2, ((1 << 63) * world + world * (world - 1) // 2) % (1 << 64),
                (U64MAX * world) % (1 << 64)]
    for r in range(world):
        assert out[r]["min"] == want_min
        assert out[r]["max"] == want_max
        assert out[r]["sum"] == want_sum
        assert out[r]["consensus"] == [12345, 0, 1]
        assert out[r]["mine_rc"] == _lib.POW_EINVAL
        assert out[r]["info"] == {"comm_count": world, "comm_device": -1}  # no context: no device


def test_custom_group_rank_count_mismatch():
    """A group whose ranks disagree on its size fails to form: the joining
    barrier counts the ranks that called it (one process, world 1, told 2)."""
    import ctypes

    from mpi_blockchain_amd import _lib

    L = _lib.load()
    calls = []

    def red(_u, vals, n, op):
        calls.append((n, op, vals[0]))
        return 0  # a "reduction" over the one rank that is really there

    fn = _lib.REDUCE_FN(red)
    g = ctypes.c_void_p()
    assert L.pow_group_init_custom(None, 2, 0, fn, None, None, ctypes.byref(g)) == _lib.POW_ECOMM and not g
    assert calls == [(1, _lib.POW_REDUCE_SUM, 1)]
    assert b"1 ranks joined a group of 2" in L.pow_last_error()
    # a failing reduction is POW_ECOMM; a null reduction or a bad rank is POW_EINVAL
    fail = _lib.REDUCE_FN(lambda *a: 1)
    assert L.pow_group_init_custom(None, 1, 0, fail, None, None, ctypes.byref(g)) == _lib.POW_ECOMM and not g
    assert L.pow_group_init_custom(None, 1, 0, _lib.REDUCE_FN(), None, None, ctypes.byref(g)) == _lib.POW_EINVAL
    assert L.pow_group_init_custom(None, 1, 1, fn, None, None, ctypes.byref(g)) == _lib.POW_EINVAL


_RCCL_PROBE = r"""
import ctypes, json, sys
from mpi_blockchain_amd import _lib
from mpi_blockchain_amd.shard import loaded_rccl_files, rccl_path
if sys.argv[1] == "torch":  # _lib.load imports torch first (libtorch_hip loads torch/lib/librccl.so)
    libs = [_lib.load(), _lib.load(test_hooks=True)]
else:  # a C caller without torch: the bare libraries
    libs = [ctypes.CDLL(_lib.LIB_PATH), ctypes.CDLL(_lib.TEST_LIB_PATH)]
    for L in libs:
        L.pow_group_rccl_path.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
before = loaded_rccl_files()
out = {"before": before, "shipped": rccl_path(libs[0]), "test": rccl_path(libs[1]), "after": loaded_rccl_files(),
       "torch": "torch" in sys.modules}
print(json.dumps(out))
"""


@pytest.mark.parametrize("first", ["torch", "alone"])
def test_group_binds_the_loaded_rccl(first):
    """One RCCL runtime per process: pow_group binds the copy the process has
    already loaded (torch's torch/lib/librccl.so, which libtorch_hip pulls in
    at import) instead of mapping /opt/rocm's beside it; a process without
    one loads librccl.so.1 from the search path.  Both libraries agree, and
    exactly one librccl file is mapped afterwards.  No GPU needed."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-c", _RCCL_PROBE, first], cwd=root, capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["shipped"] == out["test"] and out["after"] == [out["shipped"]], out
    if first == "torch":
        assert out["torch"] and out["before"] == [out["shipped"]] and "/torch/lib/" in out["shipped"], out
    else:
        assert not out["torch"] and out["before"] == [] and out["shipped"].startswith("/opt/rocm"), out


def test_native_partition_matches():
    """pow_group_partition (C ABI, used by pow_group_mine) == shard.partition."""
    from mpi_blockchain_amd.shard import native_partition

    for count in (0, 1, 7, 62, 1000, 2**32 + 3, 2**40 + 17):
        for world in (1, 2, 3, 4, 8):
            for r in range(world):
                assert native_partition(100, count, r, world) == partition(100, count, r, world)


def test_group_unique_id_and_arg_checks():
    """RCCL loads on demand (no GPU needed for the id); bad arguments are
    rejected before any RCCL or HIP call."""
    import ctypes

    from mpi_blockchain_amd import _lib
    from mpi_blockchain_amd.shard import RcclGroup

    a, b = RcclGroup.make_unique_id(), RcclGroup.make_unique_id()
    assert len(a) == len(b) == _lib.GROUP_ID_BYTES and a != b
    L = _lib.load()
    g = ctypes.c_void_p()
    assert L.pow_group_init(None, 1, 0, a, ctypes.byref(g)) == _lib.POW_EINVAL and not g
    assert L.pow_group_unique_id(None) == _lib.POW_EINVAL
    blk = _lib.Block()
    assert L.pow_group_mine(None, ctypes.byref(blk), 0, 1, 0, 9, None, 0, ctypes.byref(blk), None, None) \
        == _lib.POW_EINVAL
    assert L.pow_group_allreduce_u64(None, None, 0, 0) == _lib.POW_EINVAL


def test_board_host_protocol():
    """The stop board's host side (no GPU): slots tagged per search, the
    lowest peer counter, stale tags ignored, argument checks."""
    from mpi_blockchain_amd import _lib
    from mpi_blockchain_amd.miner import StopBoard

    with StopBoard(4) as b:
        assert b.peek(0, 1) is None  # fresh page: tag 0 everywhere
        b.post(1, 1, 500)
        b.post(2, 1, 300)
        b.post(3, 2, 100)            # another search's tag
        assert b.peek(0, 1) == 300 and b.peek(2, 1) == 500 and b.peek(0, 2) == 100
        b.post(2, 1, None)           # "nothing found yet"
        assert b.peek(0, 1) == 500
        b.post(1, 1, 62**9 - 1)      # the largest counter fits the 54-bit field
        assert b.peek(0, 1) == 62**9 - 1
        with pytest.raises(_lib.PowError):
            b.post(4, 1, 0)          # no such slot
        with pytest.raises(_lib.PowError):
            b.post(0, 0, 0)          # tag 0 is reserved (a fresh page)
        with pytest.raises(_lib.PowError):
            b.post(0, 1024, 0)
    L = _lib.load()
    import ctypes
    p = ctypes.c_void_p()
    assert L.pow_board_open(None, 0, ctypes.byref(p)) == _lib.POW_EINVAL
    assert L.pow_board_open(None, 65, ctypes.byref(p)) == _lib.POW_EINVAL
    assert L.pow_board_open(b"no-slash", 2, ctypes.byref(p)) == _lib.POW_EINVAL
    assert L.pow_board_bind(None, None, 0, 1) == _lib.POW_EINVAL


def _board_worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mpi_blockchain_amd.miner import StopBoard

    import uuid

    obj = [f"/pow_board_cputest_{os.getpid()}_{uuid.uuid4().hex[:8]}" if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    b = StopBoard(world, obj[0])
    dist.barrier()
    b.unlink()  # both mapped: the name can go, the page stays shared
    seen = []
    for tag in (1, 2):
        b.post(rank, tag, None)
        dist.barrier()
        seen.append(b.peek(rank, tag))       # nobody found anything yet
        dist.barrier()
        if rank == 1:
            b.post(1, tag, 1000 * tag + 7)   # rank 1's hit
        dist.barrier()
        seen.append(b.peek(rank, tag))
        seen.append(b.peek(rank, 3 - tag))   # the other search's tag: stale or absent
        dist.barrier()
    q.put((rank, seen))
    b.close()
    dist.destroy_process_group()


def test_board_named_world2():
    """Two processes (gloo world 2) share a named board: rank 1's post is
    what rank 0 peeks, per search tag; the name is unlinked after both mapped
    it.  The GPU side (kernels polling it) is tests/test_board_gpu.py."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_board_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # rank 0: search 1: none, then 1007 (search 2's tag: absent); search 2: none, then
    # 2007, and search 1's value is gone (one slot per rank holds the current search)
    assert out[0] == [None, 1007, None, None, 2007, None]
    assert out[1] == [None, None, None, None, None, None]  # its own slot is excluded
