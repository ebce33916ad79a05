"""The sharded search pow_group_* on the GPU (BASELINE config 4).

The C++ rounds, the stop board and the {counter, go, ok} consensus of
csrc/pow_group.cpp run here with 1, 2 and 4 ranks.  RCCL refuses two ranks on
one device and this pool gives one GPU per call, so the multi-rank tests run
every rank as its own process with its own pow_ctx on the one GPU, and the
one all-reduce per round goes over
  * pow_group_init_custom + torch.distributed gloo (ShardedMiner), or
  * pow_group_init itself, whose RCCL calls the test library
    (libpow_gpu_test.so) routes to a shared-memory stand-in
    (tests/stub_rccl): the id-derived board name, open-before-init,
    unlink-after-init and the device staging of the operand all run.
Real RCCL (pow_group_init) runs at world size 1 below; the 8-GPU run is the
driver's.

Expected values are golden (tests/golden/fingerprints_2p32.json):
S0's first solutions at d = 13, 21, 25 are 6399, 2392323 and 73523910."""
import os
import socket

import pytest

from mpi_blockchain_amd.block import make_block

pytestmark = pytest.mark.gpu

S1_PREV = b"007384e324711d0c9fab8d3ed9b7be265575e29bde9a9ea56b1d86672ee927e8"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_sharded_world1_equals_unsharded():
    """One rank: pow_group_mine over the custom (gloo) reduction returns
    exactly pow_mine's lowest counter, nonce and hash, for adaptive rounds,
    small unaligned rounds and one big round."""
    import torch.distributed as dist

    from mpi_blockchain_amd.miner import GpuMiner
    from mpi_blockchain_amd.shard import ShardedMiner

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        with GpuMiner(0) as m, ShardedMiner(m, 0, 1) as sm:
            b = make_block(7, 3, 9, 1760572800, S1_PREV)
            for d, rs in ((9, 0), (13, 5000), (17, 1 << 20), (13, 0)):
                want = m.mine(b, 300, 1 << 24, d)
                got = sm.mine(b, 300, 1 << 24, d, round_size=rs)
                assert want is not None and got is not None and got.counter == want.counter
                assert bytes(got.block.nonce) == bytes(want.block.nonce)
                assert bytes(got.block.block_hash) == bytes(want.block.block_hash)
            assert sm.mine(b, 0, 263, 9) is None  # golden: the first S1 solution is 263
    finally:
        dist.destroy_process_group()


def _fnv1a(data: bytes) -> int:
    h = 1469598103934665603
    for x in data:
        h = ((h ^ x) * 1099511628211) & ((1 << 64) - 1)
    return h


def _group_rank(rank, world, port, q, fault_rank, transport="gloo"):
    """One rank of a multi-process group on the one GPU.  transport "gloo":
    pow_group_init_custom over torch.distributed (ShardedMiner); "rccl_stub":
    pow_group_init itself, its RCCL calls served by the test library's
    stand-in (tests/stub_rccl, POW_TEST_RCCL_LIB)."""
    import ctypes
    import threading
    import time

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if rank == fault_rank:
        os.environ["POW_FAULT_INJECT"] = "mine"  # every pow_mine of this rank's context fails
    stub = transport == "rccl_stub"
    if stub:
        from mpi_blockchain_amd.build import STUB_LIB

        os.environ["POW_TEST_RCCL_LIB"] = STUB_LIB
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mpi_blockchain_amd._lib import PowError
    from mpi_blockchain_amd.miner import GpuMiner, block_hex
    from mpi_blockchain_amd.shard import RcclGroup, ShardedMiner

    out = {}
    S0 = make_block(1, 0, 9, 1700000000, b"")

    def res(r):
        return None if r is None else (r.counter, bytes(r.block.nonce).rstrip(b"\0").decode(), block_hex(r.block),
                                       r.hashes)

    def make_group(m):
        if not stub:
            return ShardedMiner(m, rank, world)
        # pow_group_init as a C caller uses it: rank 0's id (the stub's
        # ncclGetUniqueId) reaches every rank, all join ncclCommInitRank
        obj = [RcclGroup.make_unique_id(m.L) if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        g = RcclGroup(m, rank, world, obj[0])
        # the board (named after the id) was opened before the communicator
        # and unlinked once it joined, and the stub's segment is gone too
        h = _fnv1a(obj[0])
        out["shm_left"] = [p for p in (f"/dev/shm/pow_board_{h:016x}", f"/dev/shm/pow_stub_rccl_{h:016x}")
                           if os.path.exists(p)]
        return g

    # the contexts come from the test library where a test switch is needed
    # (POW_FAULT_INJECT on the faulty rank; the RCCL stand-in on every rank)
    with GpuMiner(0, test_hooks=stub or rank == fault_rank) as m:
        m.warmup()
        with make_group(m) as sm:
            out["info"] = sm.info()  # RCCL's (here the stand-in's) ncclCommCount / ncclCommCuDevice
            if fault_rank >= 0:
                try:
                    sm.mine(S0, 0, 1 << 30, 21)
                    out["fault"] = None
                except PowError as e:
                    out["fault"] = (e.code, str(e))
            else:
                # lowest mode: golden first solutions, adaptive rounds
                out["d21"] = res(sm.mine(S0, 0, 1 << 26, 21))
                out["d25"] = res(sm.mine(S0, 0, 1 << 28, 25))
                # small unaligned fixed rounds (several rounds before the hit)
                out["d13_rounds"] = res(sm.mine(S0, 300, 1 << 20, 13, round_size=1000 * world + 7))
                # nothing in range: every rank returns None
                out["none"] = res(sm.mine(S0, 0, 238, 9))
                # any-mode: one agreed solving counter
                r = sm.mine(S0, 0, 1 << 40, 28, any_solution=True)
                out["any"] = res(r)
                out["any_solves"] = r is not None and m.mine(S0, r.counter, 1, 28) is not None
                # cancellation on ONE rank (mid-search, in-flight) stops every rank;
                # the epoch is taken before the timer can move it
                ep = m.epoch
                if rank == world - 1:
                    threading.Timer(0.2, m.cancel).start()
                t = time.perf_counter()
                out["cancel"] = res(sm.mine(S0, 0, 1 << 36, 64, epoch=ep))
                out["cancel_s"] = time.perf_counter() - t
                # and the group still mines correctly afterwards
                out["after_cancel"] = res(sm.mine(S0, 0, 1 << 26, 21))
    if stub:
        out["stub_allreduces"] = ctypes.CDLL(STUB_LIB).pow_stub_rccl_allreduce_calls()
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def _run_ranks(world, fault_rank=-1, timeout=240, transport="gloo"):
    import torch.multiprocessing as mp

    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_group_rank, args=(r, world, port, q, fault_rank, transport)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        out = dict(q.get(timeout=timeout) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.exitcode is None:
                p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return out


@pytest.mark.parametrize("transport", ["gloo", "rccl_stub"])
@pytest.mark.parametrize("world", [2, 4])
def test_group_multiprocess(world, transport):
    """pow_group_mine / pow_group_mine_any with `world` peer processes (C++
    rounds, stop board shared through POSIX shared memory, the 24-byte
    consensus): every rank returns the golden lowest counter with its nonce
    and hash; any-mode agrees on one solving counter; one rank's cancel makes
    every rank return None.  transport "gloo": pow_group_init_custom over
    torch.distributed; "rccl_stub": pow_group_init's RCCL leg itself (board
    named after the id, opened before ncclCommInitRank and unlinked after it,
    d_buf/h_buf staging around ncclAllReduce), with the test library's
    shared-memory stand-in for RCCL, which refuses two ranks on one GPU."""
    from mpi_blockchain_amd.block import nonce_from_counter, solves_problem

    out = _run_ranks(world, transport=transport)
    # the group as its transport sees it: `world` ranks, each communicator on device 0
    assert all(out[r]["info"] == {"comm_count": world, "comm_device": 0} for r in range(world)), out
    if transport == "rccl_stub":
        for r in range(world):
            assert out[r]["shm_left"] == [], out[r]["shm_left"]
            # every one of the 7 group searches above ends its rounds with the stand-in's all-reduce
            assert out[r]["stub_allreduces"] >= 7, out[r]["stub_allreduces"]
    for key, ctr, d in (("d21", 2392323, 21), ("d25", 73523910, 25), ("d13_rounds", 6399, 13)):
        vals = {out[r][key][:3] for r in range(world)}
        assert len(vals) == 1, (key, vals)  # the same result on every rank
        c, nonce, hx = vals.pop()
        assert c == ctr and nonce == nonce_from_counter(ctr).rstrip(b"\0").decode(), (key, c, nonce)
        assert solves_problem(hx, d) and not solves_problem(hx, 64)
    assert all(out[r]["none"] is None for r in range(world))
    anys = {out[r]["any"][:3] for r in range(world)}
    assert len(anys) == 1 and all(out[r]["any_solves"] for r in range(world))
    assert all(out[r]["cancel"] is None for r in range(world))
    # the first round is 2^30 counters per rank (~0.13 s alone, world x that on one
    # shared GPU); the whole 2^36 range would take ~8 s
    assert all(out[r]["cancel_s"] < 0.5 + 0.3 * world for r in range(world)), [out[r]["cancel_s"] for r in out]
    assert all(out[r]["after_cancel"][0] == 2392323 for r in range(world))


@pytest.mark.parametrize("transport", ["gloo", "rccl_stub"])
def test_group_failure_propagates(transport):
    """An injected failure on one rank (POW_FAULT_INJECT=mine in the test
    library, libpow_gpu_test.so: its pow_mine returns POW_EHIP) makes every rank's pow_group_mine fail together: the
    failing rank with its own error, its peers with POW_ECOMM."""
    from mpi_blockchain_amd._lib import POW_ECOMM, POW_EHIP

    world = 2
    out = _run_ranks(world, fault_rank=1, transport=transport)
    assert out[1]["fault"][0] == POW_EHIP and "injected fault" in out[1]["fault"][1]
    assert out[0]["fault"][0] == POW_ECOMM and "a peer rank failed" in out[0]["fault"][1]


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


def test_native_group_beside_torch_rccl():
    """bench.py at N > 1 runs torch's nccl (RCCL) process group and the
    library's own RCCL communicator (pow_group, RCCL dlopen'ed) in one
    process: both on this GPU at world size 1, collectives on each, then a
    group search.  pow_group binds the RCCL copy torch loaded (one RCCL
    runtime in the process), and RCCL's own view of the communicator
    (ncclCommCount, ncclCommCuDevice) is one rank on device 0."""
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
        from mpi_blockchain_amd.shard import loaded_rccl_files, rccl_path

        with GpuMiner(0) as m, RcclGroup.from_torch(m) as g:
            assert g.info() == {"comm_count": 1, "comm_device": 0}
            files = loaded_rccl_files()
            assert len(files) == 1 and rccl_path(m.L) == files[0] and "torch" in files[0], (files, rccl_path(m.L))
            assert g.allreduce([9, 2], "min") == [9, 2]
            r = g.mine(make_block(1, 0, 9, 1700000000, b""), 0, 1 << 20, 9)
            assert r is not None and r.counter == 238
            dist.all_reduce(t)  # torch's communicator still works beside ours
            assert t.sum().item() == 4
    finally:
        dist.destroy_process_group()


LONELY_TORCH_RCCL = r"""
import sys, time
sys.path.insert(0, %r)
import torch  # torch's RCCL (2.26.6 on this image) is the one pow_group binds, as in bench.py
from mpi_blockchain_amd._lib import PowError
from mpi_blockchain_amd.block import make_block
from mpi_blockchain_amd.miner import GpuMiner
from mpi_blockchain_amd.shard import RcclGroup, rccl_path
with GpuMiner(0) as m:
    print("rccl", rccl_path(m.L), flush=True)
    t = time.monotonic()
    try:
        RcclGroup(m, 0, 2, RcclGroup.make_unique_id(m.L), timeout_ms=3000)
        print("joined?!", flush=True)
    except PowError as e:
        print(f"lonely: {time.monotonic() - t:.3f} s: {e}", flush=True)
    with RcclGroup(m, 0, 1, RcclGroup.make_unique_id(m.L)) as g:
        assert g.allreduce([5, 7], "min") == [5, 7]
        r = g.mine(make_block(1, 0, 9, 1700000000, b""), 0, 1 << 32, 21)
        print("one-rank group counter", r.counter, flush=True)
print("ok", flush=True)
"""


def test_group_init_deadline_torch_rccl():
    """pow_group_init's join deadline with torch's own RCCL, the copy bench.py's
    ranks bind (2.26.6 honours the non-blocking config, unlike /opt/rocm's
    2.27.7 that tests/test_c_consumer.py::test_group_init_deadline[rccl]
    covers): rank 0 of a 2-rank group whose peer never joins gets POW_ECOMM
    after its 3 s deadline, and the same context then forms a one-rank group
    that mines S0 at d = 21 to its golden lowest counter."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run(["timeout", "-k", "5", "120", sys.executable, "-c", LONELY_TORCH_RCCL % root],
                       capture_output=True, text=True)
    assert p.returncode == 0, p.stdout + p.stderr[-3000:]
    assert "torch/lib/librccl.so" in p.stdout, p.stdout
    line = next(ln for ln in p.stdout.splitlines() if ln.startswith("lonely: "))
    assert "POW_ECOMM" in line and "rank 0 of 2" in line and "not every rank joined within 3.000 s" in line, line
    assert 2.9 < float(line.split()[1]) < 8.0, line
    assert "one-rank group counter 2392323" in p.stdout and p.stdout.rstrip().endswith("ok"), p.stdout


TWO_RANKS_ONE_GPU = r"""
import os, sys, time
sys.path.insert(0, %r)
import torch  # torch's RCCL, as bench.py's ranks bind it
from mpi_blockchain_amd._lib import PowError
from mpi_blockchain_amd.miner import GpuMiner
from mpi_blockchain_amd.shard import RcclGroup
rank, idf = int(sys.argv[1]), sys.argv[2]
with GpuMiner(0) as m:
    if rank == 0:
        open(idf + ".tmp", "wb").write(RcclGroup.make_unique_id(m.L))
        os.replace(idf + ".tmp", idf)
    while not os.path.exists(idf):
        time.sleep(0.01)
    uid = open(idf, "rb").read()
    t = time.monotonic()
    try:
        RcclGroup(m, rank, 2, uid, timeout_ms=20000).close()
        print(f"rank {rank}: joined", flush=True)
    except PowError as e:
        print(f"rank {rank}: {time.monotonic() - t:.3f} s: {e}", flush=True)
"""


def test_real_rccl_two_ranks_one_gpu_fail_fast(tmp_path):
    """Two processes join one real-RCCL group (torch's copy) on the one GPU of
    the box: RCCL's bootstrap connects them, then RCCL refuses two ranks on one
    device.  Neither rank hangs: each pow_group_init returns POW_ECOMM, either
    with RCCL's own error or at its 20 s deadline, and both processes exit 0.
    This is the only multi-process run of RCCL itself a one-GPU box allows."""
    import subprocess
    import sys
    import time

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    idf = str(tmp_path / "id")
    t = time.monotonic()
    procs = [subprocess.Popen(["timeout", "-k", "5", "90", sys.executable, "-c", TWO_RANKS_ONE_GPU % root, str(r), idf],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = [p.communicate(timeout=120) for p in procs]
    wall = time.monotonic() - t
    for r, (p, (out, err)) in enumerate(zip(procs, outs)):
        print(out.strip())
        assert p.returncode == 0, (r, out, err[-3000:])
        line = next(ln for ln in out.splitlines() if ln.startswith(f"rank {r}: "))
        assert "POW_ECOMM" in line and f"rank {r} of 2 on HIP device 0" in line, line
        assert float(line.split()[2]) < 26.0, line
    assert wall < 90, wall


BROKEN_GROUP = r"""
import os, sys, time
sys.path.insert(0, %r)
rank, idf, case, stub = int(sys.argv[1]), sys.argv[2], sys.argv[3], sys.argv[4]
os.environ.update(POW_TEST_RCCL_LIB=stub, POW_STUB_TIMEOUT_S="3")
if case == "wedged" and rank == 1:  # this rank's launches stall 300 ms behind a 30 ms watchdog
    os.environ.update(POW_TEST_STALL_US="300000", POW_WATCHDOG_MS="30")
from mpi_blockchain_amd._lib import PowError
from mpi_blockchain_amd.block import make_block
from mpi_blockchain_amd.miner import GpuMiner
from mpi_blockchain_amd.shard import RcclGroup
S0 = make_block(1, 0, 9, 1700000000, b"")
m = GpuMiner(0, test_hooks=True)
if rank == 0:
    open(idf + ".tmp", "wb").write(RcclGroup.make_unique_id(m.L))
    os.replace(idf + ".tmp", idf)
while not os.path.exists(idf):
    time.sleep(0.01)
g = RcclGroup(m, rank, 2, open(idf, "rb").read(), timeout_ms=30000)
print(f"rank {rank}: joined", flush=True)
if case == "exits" and rank == 1:
    os._exit(0)  # dies once the group has formed
t = time.monotonic()
try:
    # d = 21: the first launch of each shard is the latency kernel K1', whose watchdog (30 ms +
    # 2 ns per counter) the wedged rank's 300 ms stall outlasts; rank 0 finds S0's 2392323 at once
    r = g.mine(S0, 0, 1 << 40, 21, any_solution=True)
    print(f"rank {rank}: mined?! {r}", flush=True)
except PowError as e:
    print(f"rank {rank}: mine failed after {time.monotonic() - t:.3f} s: {e}", flush=True)
try:
    g.allreduce([1], "sum")
    print(f"rank {rank}: allreduce ok?!", flush=True)
except PowError as e:
    print(f"rank {rank}: allreduce after: {e}", flush=True)
t = time.monotonic()
g.close()
print(f"rank {rank}: close {time.monotonic() - t:.3f} s", flush=True)
if not (case == "wedged" and rank == 1):  # a context whose watchdog fired is not reused
    print(f"rank {rank}: after {m.mine(S0, 0, 1 << 32, 21).counter}", flush=True)
m.close()
print(f"rank {rank}: ok", flush=True)
"""


def _field(out: str, rank: int, key: str) -> str:
    return next(ln for ln in out.splitlines() if ln.startswith(f"rank {rank}: {key}"))


@pytest.mark.parametrize("case", ["exits", "wedged"])
def test_group_broken_fails_every_rank_fast(tmp_path, case):
    """A group whose round cannot complete, through pow_group_init's
    RCCL leg with the stand-in (its barrier gives up after 3 s here, as a
    stand-in for pow_group's own deadline on RCCL's asynchronous all-reduce):
      exits  - rank 1 dies once the group has formed: rank 0's round-end
               all-reduce fails (POW_ECOMM);
      wedged - rank 1's launch is stuck (its watchdog fires): rank 1 returns
               its own error at once without joining the round's all-reduce,
               and rank 0's all-reduce fails at the stand-in's deadline.
    Every later collective of a broken group returns POW_ECOMM at once,
    pow_group_destroy returns (bounded drain), and a healthy context mines
    S0 at d = 21 to 2392323 afterwards."""
    import subprocess
    import sys

    from mpi_blockchain_amd.build import STUB_LIB, build_test_stub

    build_test_stub()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    idf = str(tmp_path / "id")
    procs = [subprocess.Popen(["timeout", "-k", "5", "120", sys.executable, "-c", BROKEN_GROUP % root, str(r), idf,
                               case, STUB_LIB], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for r in range(2)]
    outs = [p.communicate(timeout=150) for p in procs]
    for p, (out, err) in zip(procs, outs):
        print(out.strip())
        assert p.returncode == 0, (out, err[-3000:])
    out0, out1 = outs[0][0], outs[1][0]
    m0 = _field(out0, 0, "mine failed after")
    assert "POW_ECOMM" in m0 and "ncclAllReduce" in m0 and float(m0.split()[5]) < 15, m0
    assert "the group is broken" in _field(out0, 0, "allreduce after")
    assert float(_field(out0, 0, "close").split()[3]) < 10
    assert _field(out0, 0, "after") == "rank 0: after 2392323" and "rank 0: ok" in out0
    if case == "exits":
        assert "rank 1: joined" in out1 and "rank 1: mine" not in out1
    else:
        m1 = _field(out1, 1, "mine failed after")
        assert "POW_EHIP" in m1 and "watchdog" in m1 and "did not join the round's all-reduce" in m1, m1
        assert float(m1.split()[5]) < 5, m1  # at once: not after the stand-in's 3 s or a round's shard
        assert "the group is broken" in _field(out1, 1, "allreduce after")
        assert float(_field(out1, 1, "close").split()[3]) < 15 and "rank 1: ok" in out1
