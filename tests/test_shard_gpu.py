"""ShardedMiner on the GPU: pow_mine per shard + the torch.distributed
all-reduce(min) (gloo here, world size 1; RCCL in bench.py) returns the same
counter as one un-sharded pow_mine."""
import os
import socket

import pytest

from mpi_blockchain_amd.block import make_block

pytestmark = pytest.mark.gpu


def test_sharded_equals_unsharded():
    import torch.distributed as dist

    from mpi_blockchain_amd.miner import GpuMiner
    from mpi_blockchain_amd.shard import ShardedMiner, sharded_mine

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        with GpuMiner(0) as m:
            b = make_block(7, 3, 9, 1760572800, b"007384e324711d0c9fab8d3ed9b7be265575e29bde9a9ea56b1d86672ee927e8")
            sm = ShardedMiner(m, 0, 1)
            for d in (9, 13, 17):
                want = m.mine(b, 0, 1 << 24, d)
                got = sm.mine(b, 0, 1 << 24, d, round_size=1 << 20)
                assert want is not None and got == want.counter
            # 3 simulated ranks over the same range, each mining its shard on the GPU
            def search(start, n):
                r = m.mine(b, start, n, 13)
                return None if r is None else r.counter
            from mpi_blockchain_amd.shard import NONE, partition
            best = NONE
            for rank in range(3):
                v = sharded_mine(search, lambda x: x, 0, 1 << 20, 1 << 20, rank, 3)
                best = min(best, NONE if v is None else v)
            assert best == m.mine(b, 0, 1 << 20, 13).counter
    finally:
        dist.destroy_process_group()


def test_native_group_world1():
    """pow_group_mine (C++ rounds + RCCL all-reduce) on one rank returns
    exactly pow_mine's lowest counter, for one round and for many small
    rounds; the all-reduce itself; cancellation."""
    from mpi_blockchain_amd.miner import GpuMiner
    from mpi_blockchain_amd.shard import RcclGroup

    with GpuMiner(0) as m:
        with RcclGroup(m, 0, 1, RcclGroup.make_unique_id()) as g:
            assert g.allreduce([5, 7, 1 << 63], "min") == [5, 7, 1 << 63]
            assert g.allreduce([3, 4], "sum") == [3, 4]
            b = make_block(7, 3, 9, 1760572800, b"007384e324711d0c9fab8d3ed9b7be265575e29bde9a9ea56b1d86672ee927e8")
            for d, rs in ((9, 0), (13, 1 << 12), (17, 1 << 20), (13, 5000)):
                want = m.mine(b, 300, 1 << 24, d)
                got = g.mine(b, 300, 1 << 24, d, round_size=rs)
                assert want is not None and got is not None
                assert got.counter == want.counter
                assert bytes(got.block.nonce) == bytes(want.block.nonce)
                assert bytes(got.block.block_hash) == bytes(want.block.block_hash)
            assert g.mine(b, 0, 263, 9) is None  # golden: the first S1 solution is 263
            assert g.mine(b, 0, 264, 9, round_size=100).counter == 263
            m.cancel()
            assert g.mine(b, 0, 1 << 40, 60, epoch=(m.epoch - 1) & 0xFFFFFFFF) is None


def test_native_group_from_torch():
    """RcclGroup.from_torch: the RCCL id travels over torch.distributed."""
    import torch.distributed as dist

    from mpi_blockchain_amd.miner import GpuMiner
    from mpi_blockchain_amd.shard import RcclGroup

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        with GpuMiner(0) as m, RcclGroup.from_torch(m) as g:
            b = make_block(1, 0, 9, 1700000000, b"")
            r = g.mine(b, 0, 1 << 20, 9)
            assert r is not None and r.counter == 238  # golden: first S0 solution
    finally:
        dist.destroy_process_group()


def _board_rank(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), POW_GRID_PER_CU="4")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mpi_blockchain_amd.miner import GpuMiner
    from mpi_blockchain_amd.shard import ShardedMiner

    out = {}
    with GpuMiner(0) as m:
        m.warmup()
        sm = ShardedMiner(m, rank, world, board=True)
        b = make_block(1, 0, 9, 1700000000, b"")
        # lowest mode: S0's first d = 21 solution (golden) lies in rank 0's shard of
        # the first 2^26-counter round; rank 1's shard stops on rank 0's hit
        out["lowest"] = sm.mine(b, 0, 1 << 26, 21, round_size=1 << 26)
        # any-mode: the first solution either rank finds; both agree on it
        out["any"] = sm.mine(b, 0, 1 << 40, 28, any_solution=True)
        out["any_solves"] = m.mine(b, out["any"], 1, 28) is not None if out["any"] is not None else False
        sm.close()
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_board_two_ranks():
    """Two processes share this GPU (gloo; RCCL would refuse two ranks on one
    device), each a ShardedMiner rank with a named stop board: the lowest
    counter is the golden one on both ranks, and an any-mode search ends
    with one agreed, solving counter."""
    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_board_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        out = dict(q.get(timeout=180) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert out[0]["lowest"] == out[1]["lowest"] == 2392323
    assert out[0]["any"] == out[1]["any"] is not None
    assert out[0]["any_solves"] and out[1]["any_solves"]


def test_native_group_beside_torch_rccl():
    """bench.py at N > 1 runs torch's nccl (RCCL) process group and the
    library's own RCCL communicator (pow_group, RCCL dlopen'ed) in one
    process: both on this GPU at world size 1, collectives on each, then a
    group search."""
    import torch
    import torch.distributed as dist

    from mpi_blockchain_amd.miner import GpuMiner
    from mpi_blockchain_amd.shard import RcclGroup

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        t = torch.ones(4, device="cuda:0")
        dist.all_reduce(t)
        assert t.sum().item() == 4
        with GpuMiner(0) as m, RcclGroup.from_torch(m) as g:
            assert g.allreduce([9, 2], "min") == [9, 2]
            r = g.mine(make_block(1, 0, 9, 1700000000, b""), 0, 1 << 20, 9)
            assert r is not None and r.counter == 238
            dist.all_reduce(t)  # torch's communicator still works beside ours
            assert t.sum().item() == 4
    finally:
        dist.destroy_process_group()
