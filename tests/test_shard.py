"""Sharded search logic (mpi_blockchain_amd/shard.py), CPU only: static
partition, min-counter winner, and a real world_size-2 run over
torch.distributed gloo (the same all-reduce(MIN) code path the GPU ranks use
over RCCL).  The per-rank search is the CPU oracle here — this tests the
sharding and the collective, not the kernel."""
import os
import socket

import pytest

from mpi_blockchain_amd.shard import NONE, partition, sharded_mine
from oracle.oracle import Oracle, make_oblock


def test_partition_covers_range():
    for count in (0, 1, 7, 62, 1000, 2**32 + 3):
        for world in (1, 2, 3, 4, 8):
            parts = [partition(100, count, r, world) for r in range(world)]
            assert parts[0][0] == 100
            for (s0, n0), (s1, _) in zip(parts, parts[1:]):
                assert s0 + n0 == s1
            assert sum(n for _, n in parts) == count


def _simulated_world(search, start, count, round_size, world):
    """Run every rank's search per round and reduce by hand (what RCCL does)."""
    done = 0
    while done < count:
        n = min(round_size, count - done)
        best = NONE
        for r in range(world):
            s, k = partition(start + done, n, r, world)
            v = search(s, k) if k else None
            best = min(best, NONE if v is None else v)
        if best != NONE:
            return best
        done += n
    return None


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_sharded_equals_single(world):
    O = Oracle()
    b = make_oblock(1, 0, 9, 1700000000, b"")

    def search(s, n):
        return O.mine(b, s, n, 13)

    single = O.mine(b, 0, 1 << 15, 13)
    # the first solution at d = 13 is 6399
    assert single == 6399
    for rs in (1000, 4096, 1 << 15):
        assert _simulated_world(search, 0, 1 << 15, rs, world) == single
    # rank-local view through sharded_mine with a fake reduction
    calls = []

    def fake_min(v):
        calls.append(v)
        return v

    got = sharded_mine(search, fake_min, 6000, 1000, 1000, 0, 1)
    assert got == 6399 and calls == [6399]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mpi_blockchain_amd.shard import torch_allreduce_min

    O = Oracle()
    b = make_oblock(7, 3, 9, 1760572800, b"007384e324711d0c9fab8d3ed9b7be265575e29bde9a9ea56b1d86672ee927e8")
    red = torch_allreduce_min()
    res = []
    for start, count, rs, d in ((0, 1 << 12, 1 << 12, 9), (300, 5000, 2048, 9), (0, 40000, 8192, 13),
                                (0, 40000, 0, 13)):  # rs 0: adaptive rounds (round_plan)
        res.append(sharded_mine(lambda s, n: O.mine(b, s, n, d), red, start, count, rs, rank, world, d))
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    O = Oracle()
    b = make_oblock(7, 3, 9, 1760572800, b"007384e324711d0c9fab8d3ed9b7be265575e29bde9a9ea56b1d86672ee927e8")
    want = [O.mine(b, 0, 1 << 12, 9), O.mine(b, 300, 5000, 9), O.mine(b, 0, 40000, 13), O.mine(b, 0, 40000, 13)]
    assert want[0] == 263  # golden: first S1 solution
    assert out[0] == out[1] == want


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


def test_round_plan_adaptive():
    """Adaptive rounds (round_size 0): first round ~4x the expected trials,
    at least 2^16 per rank, growing 4x up to 2^30 per rank; the winner equals
    one search over the whole range (multi-rank: test_gloo_world2)."""
    from mpi_blockchain_amd.shard import round_plan

    assert round_plan(8, 25) == (1 << 27, 8 << 30)
    assert round_plan(2, 9) == (2 << 16, 2 << 30)
    assert round_plan(1, 60)[0] == 1 << 30
    O = Oracle()
    b = make_oblock(1, 0, 9, 1700000000, b"")
    for d in (9, 13, 17):
        sizes = []

        def search(s, n):
            sizes.append(n)
            return O.mine(b, s, n, d)
        assert sharded_mine(search, lambda v: v, 0, 1 << 20, 0, 0, 1, d) == O.mine(b, 0, 1 << 20, d)
        assert sizes[0] == round_plan(1, d)[0] and all(y == 4 * x for x, y in zip(sizes, sizes[1:-1]))


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
