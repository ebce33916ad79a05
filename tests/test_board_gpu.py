"""Cross-GPU stop board (include/pow_gpu.h): a hit of one context stops the
other contexts of the same search inside their running launches.

BASELINE config 4 asks for winner selection AND cancellation across GPUs.
These tests drive two contexts on the one GPU of the box (in one process, and
in two processes through POSIX shared memory): the mechanism is the same as
across the GPUs of a node, since every GPU reads the board over PCIe.  The
running context is created with POW_GRID_PER_CU=4 (a switch of the test
library, libpow_gpu_test.so) so that it leaves half the workgroup slots free
and the finder's launch runs beside it.
"""
import json
import os
import subprocess
import sys
import threading
import time
import uuid

import pytest

from mpi_blockchain_amd.block import make_block

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

S0 = dict(index=1, owner=0, difficulty=9, created_at=1700000000, prev=b"")
# Golden (SURVEY §8c / tests/golden/fingerprints_2p32.json): S0's first
# solving counters at d = 9 and d = 21.
FIRST_D9, FIRST_D21 = 238, 2392323


def s0():
    return make_block(S0["index"], S0["owner"], S0["difficulty"], S0["created_at"], S0["prev"])


def half_grid_miner():
    """A context of the test library (libpow_gpu_test.so) whose K1 grid is 4
    workgroups per CU (POW_GRID_PER_CU, a test-build switch)."""
    from mpi_blockchain_amd.miner import GpuMiner

    os.environ["POW_GRID_PER_CU"] = "4"
    try:
        m = GpuMiner(0, test_hooks=True)
    finally:
        del os.environ["POW_GRID_PER_CU"]
    m.warmup()
    return m


@pytest.mark.parametrize("any_solution", [True, False])
def test_board_stops_running_peer(any_solution):
    """Context B mines a range with no solution (d = 64, 2^34 counters:
    ~2 s even at the whole GPU's rate); context A then finds S0's first d = 9
    solution and its kernel publishes it.  B must stop within a few ms of A's
    return, in both modes (lowest mode: A's counter 238 is below every counter
    B would compute).  B's half grid still runs near the full rate while A is
    idle, and A's call itself takes 20-110 ms beside B, so the check is on
    B's stop time, not on a trial count tied to the sleep below."""
    from mpi_blockchain_amd.miner import GpuMiner, StopBoard

    b = s0()
    with StopBoard(2) as board, GpuMiner(0) as A, half_grid_miner() as B:
        A.warmup()
        A.bind_board(board, 0, 7)
        B.bind_board(board, 1, 7)
        res = {}

        def run_b():
            t = time.perf_counter()
            res["r"] = B.mine(b, 1 << 36, 1 << 34, 64, any_solution=any_solution)
            res["end"] = time.perf_counter()
            res["secs"] = res["end"] - t
            res["hashes"] = B.stats()["hashes"]

        th = threading.Thread(target=run_b)
        th.start()
        time.sleep(0.15)  # B's kernel is running
        ra = A.mine(b, 0, 1 << 20, 9, any_solution=any_solution)
        a_end = time.perf_counter()
        th.join(timeout=30)
        assert not th.is_alive()
        assert ra is not None
        if not any_solution:
            assert ra.counter == FIRST_D9
        assert A.mine(b, ra.counter, 1, 9) is not None  # a real solution
        assert board.peek(1, 7) is not None  # A's slot, as B sees it
        assert res["r"] is None
        lag = res["end"] - a_end
        print(f"any={any_solution}: B stopped {1e3 * lag:.3f} ms after A returned; "
              f"B ran {res['secs']:.3f} s, {res['hashes']} trials")
        assert -0.001 < lag < 0.005, lag  # B was still running when A returned, and stopped at once
        assert res["hashes"] < (1 << 34) // 2
        A.bind_board(None)
        B.bind_board(None)


def test_board_lowest_mode_is_exact():
    """Lowest mode stops only counters ABOVE a peer's solution: with a peer
    solution above this range's lowest, pow_mine still returns the exact
    lowest; with one below it, it returns None (the peer wins the
    all-reduce).  A stale tag is ignored."""
    from mpi_blockchain_amd.miner import GpuMiner, StopBoard

    b = s0()
    with StopBoard(2) as board, GpuMiner(0) as m:
        m.bind_board(board, 0, 3)
        board.post(1, 3, 3_000_000)  # above S0's first d = 21 solution
        r = m.mine(b, 0, 1 << 26, 21)
        assert r is not None and r.counter == FIRST_D21
        # slot 1 (seen from slot 0) keeps the peer's value; slot 0 holds this context's hit
        assert board.peek(0, 3) == 3_000_000 and board.peek(1, 3) == FIRST_D21
        board.post(1, 3, 1_000_000)  # below it: the rest of the range is moot
        assert m.mine(b, 0, 1 << 26, 21) is None
        m.bind_board(board, 0, 4)  # a new search: slot 1's tag-3 value is stale
        r = m.mine(b, 0, 1 << 26, 21)
        assert r is not None and r.counter == FIRST_D21
        assert board.peek(1, 4) == FIRST_D21  # published by this context (slot 0)
        m.bind_board(None)
        r = m.mine(b, 0, 1 << 26, 21)  # unbound: the board plays no part
        assert r is not None and r.counter == FIRST_D21


def test_board_shared_between_processes():
    """The same across two processes (one GPU each in a real node): a named
    board in POSIX shared memory, registered with hipHostRegister."""
    from mpi_blockchain_amd.miner import GpuMiner, StopBoard

    name = f"/pow_board_test_{os.getpid()}_{uuid.uuid4().hex[:8]}"
    env = dict(os.environ, POW_GRID_PER_CU="4")
    with StopBoard(2, name) as board, GpuMiner(0) as A:
        A.warmup()
        p = subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "board_peer.py"), name, "1", "9"],
                             stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
        try:
            line = p.stdout.readline()
            assert line.strip() == "ready", (line, p.stderr.read() if p.poll() is not None else "")
            board.unlink()  # both processes have it mapped
            A.bind_board(board, 0, 9)
            time.sleep(0.3)  # the peer's kernel is running
            ra = A.mine(s0(), 0, 1 << 20, 9, any_solution=True)
            assert ra is not None
            out, err = p.communicate(timeout=60)
        finally:
            if p.poll() is None:
                p.kill()
        assert p.returncode == 0, err[-2000:]
        res = json.loads(out.strip().splitlines()[-1])
        print("peer process:", res)
        assert res["found"] is False
        assert res["secs"] < 0.3 + 0.5, res  # not the seconds its 2^34-counter range would take
        assert res["hashes"] < 1 << 33
        A.bind_board(None)


def test_group_mine_any_world1():
    """pow_group_mine_any on one rank returns a real solution (a member of the
    golden d = 21 set) with its block hash, like pow_mine_any."""
    import json as _json

    from mpi_blockchain_amd.miner import GpuMiner, block_hex
    from mpi_blockchain_amd.shard import RcclGroup

    with open(os.path.join(ROOT, "tests", "golden", "fingerprints_2p32.json")) as f:
        first21 = _json.load(f)["ladder"]["21"]["first"]
    with GpuMiner(0) as m, RcclGroup(m, 0, 1, RcclGroup.make_unique_id()) as g:
        b = s0()
        r = g.mine(b, 0, 1 << 32, 21, any_solution=True)
        assert r is not None
        lo = m.mine(b, 0, 1 << 32, 21)
        assert r.counter >= lo.counter
        assert m.mine(b, r.counter, 1, 21).counter == r.counter  # it solves
        assert block_hex(r.block) == block_hex(m.mine(b, r.counter, 1, 0).block)
        if r.counter < first21[-1]:
            assert r.counter in first21
        # the lowest-counter group search is unchanged by the board
        assert g.mine(b, 0, 1 << 32, 21).counter == FIRST_D21


def test_bound_lowest_mode_peer_below_returns_zero():
    """ADVICE r03 / include/pow_gpu.h: with a bound board, lowest-mode pow_mine
    returns 0 whenever a peer's slot holds a counter below the one it found,
    even though its own range holds a solution; the context holding the lower
    counter returns it.  Two contexts, one board, two searches (tags), both
    orders: S1's lowest d = 9 solution is 263 and S0's is 238 (golden)."""
    from mpi_blockchain_amd.miner import GpuMiner, StopBoard

    s1 = make_block(7, 3, 9, 1760572800, b"007384e324711d0c9fab8d3ed9b7be265575e29bde9a9ea56b1d86672ee927e8")
    with StopBoard(2) as board, GpuMiner(0) as A, GpuMiner(0) as B:
        for tag in (11, 12):
            A.bind_board(board, 0, tag)
            B.bind_board(board, 1, tag)
            if tag == 11:  # the lower one first: it returns its counter; the higher one then returns 0
                rb = B.mine(s0(), 0, 1 << 16, 9)
                ra = A.mine(s1, 0, 1 << 16, 9)
                assert rb is not None and rb.counter == FIRST_D9
                assert ra is None
                # unbound, A's own range does hold a solution
                A.bind_board(None)
                assert A.mine(s1, 0, 1 << 16, 9).counter == 263
            else:  # the higher one first returns 263; the lower one still returns its own 238
                ra = A.mine(s1, 0, 1 << 16, 9)
                rb = B.mine(s0(), 0, 1 << 16, 9)
                assert ra is not None and ra.counter == 263
                assert rb is not None and rb.counter == FIRST_D9
                assert board.peek(1, tag) == 263 and board.peek(0, tag) == FIRST_D9
        A.bind_board(None)
        B.bind_board(None)


def sentinel_idle_miner():
    """A context of the test library whose K1 mine launches keep the sentinel
    wave (workgroup 0, wave 0) out of the work queue from the start
    (POW_TEST_SENTINEL_IDLE), and whose pow_mine skips the latency kernel
    (POW_LAT_MAX=0), so every launch is K1."""
    from mpi_blockchain_amd.miner import GpuMiner

    os.environ.update(POW_TEST_SENTINEL_IDLE="1", POW_LAT_MAX="0")
    try:
        m = GpuMiner(0, test_hooks=True)
    finally:
        del os.environ["POW_TEST_SENTINEL_IDLE"], os.environ["POW_LAT_MAX"]
    m.warmup()
    return m


@pytest.mark.parametrize("any_solution", [True, False])
def test_cancel_reaches_the_grid_after_the_sentinel_is_done(any_solution):
    """the sentinel wave is the only reader of host memory, so it
    must keep polling after its own chunks are done while the rest of the grid
    still runs (pow_kernels.hip, the exit wait).  Here it takes no chunk at
    all (a test-library flag), so every poll of the launch comes from that
    wait: a cancel 30 ms into a 2^30-counter K1 launch (~0.13 s) must still
    stop it within a few ms, and a peer's hit on the board likewise.  The
    same flag leaves the results exact (golden lowest counter)."""
    from mpi_blockchain_amd.miner import StopBoard

    b = s0()
    with sentinel_idle_miner() as m:
        r = m.mine(b, 0, 1 << 26, 21, any_solution=any_solution)
        assert r is not None and (r.counter == FIRST_D21 or any_solution)
        m.cancel()  # arm the GPU-side epoch check
        ep = m.epoch
        res = {}

        def run():
            res["r"] = m.mine(b, 0, 1 << 40, 60, epoch=ep, any_solution=any_solution)
            res["t"] = time.perf_counter()

        th = threading.Thread(target=run)
        th.start()
        time.sleep(0.03)
        t_cancel = time.perf_counter()
        m.cancel()
        th.join(timeout=30)
        assert not th.is_alive() and res["r"] is None
        assert res["t"] - t_cancel < 0.02, res["t"] - t_cancel
        # a peer's hit on the board, seen only by the waiting sentinel
        with StopBoard(2) as board:
            m.bind_board(board, 0, 21)
            th = threading.Thread(target=run)
            ep = m.epoch
            th.start()
            time.sleep(0.03)
            t_post = time.perf_counter()
            board.post(1, 21, 5)  # below every counter of the range
            th.join(timeout=30)
            assert not th.is_alive() and res["r"] is None
            assert res["t"] - t_post < 0.02, res["t"] - t_post
            m.bind_board(None)
