"""GPU parity: the gfx950 path (through the C ABI) vs the reference's own
outputs (tests/golden/golden.json, generated from /root/reference's block.cpp +
picosha2.h) — bit-exact digests and identical solution SETS.

Run on an MI355X:  python -m pytest tests -m gpu -x -q
"""
import hashlib
import os
import sys

import numpy as np
import pytest

from mpi_blockchain_amd._lib import COUNTER_LIMIT, PowError
from mpi_blockchain_amd.block import block_to_str, field, make_block, nonce_from_counter
from mpi_blockchain_amd.miner import GpuMiner, block_hex, refresh_template

from helpers import block_from_random, block_from_template, with_nonce

pytestmark = pytest.mark.gpu


def fp(arr) -> str:
    return hashlib.sha256(np.asarray(arr, dtype="<u4").tobytes()).hexdigest()


@pytest.fixture(scope="module")
def miner():
    m = GpuMiner(0)
    yield m
    m.close()


def hooked_miner(**env) -> GpuMiner:
    """A context of the test library (libpow_gpu_test.so) with test switches
    set for its pow_init; the shipped library has none of them."""
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return GpuMiner(0, test_hooks=True)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def miner_full():
    """A context whose every launch uses the d > 32 kernel variant."""
    m = hooked_miner(POW_FORCE_FULL=1)
    yield m
    m.close()


@pytest.fixture(scope="module")
def miner_k1():
    """pow_mine on the throughput kernel only (latency kernel K1' disabled)."""
    m = hooked_miner(POW_LAT_MAX=0)
    yield m
    m.close()


@pytest.fixture(params=["lat+k1", "k1"])
def mminer(request, miner, miner_k1):
    return miner if request.param == "lat+k1" else miner_k1


def test_device_is_gfx950(miner):
    import re

    info = miner.device_info()
    assert info["cu_count"] > 0
    # the full PCI address the N > 1 bench's topology check compares (function included)
    assert re.fullmatch(r"[0-9a-f]{4}:[0-9a-f]{2}:[0-9a-f]{2}\.[0-7]", miner.pci_bus_id().lower()), miner.pci_bus_id()


def test_edge_counter_digests(miner, golden, templates):
    """block_to_hash on the GPU (K2) for every template x edge counter."""
    blocks, want = [], []
    for e in golden["digests"]:
        b = block_from_template(templates[e["template"]])
        n = nonce_from_counter(e["counter"])
        assert n[:9].decode() == e["nonce"]
        blocks.append(with_nonce(b, n))
        want.append(e["hex"])
    assert miner.hash_blocks(blocks) == want


def test_random_block_digests(miner, golden):
    blocks = [block_from_random(e) for e in golden["random_blocks"]]
    assert miner.hash_blocks(blocks) == [e["hex"] for e in golden["random_blocks"]]
    # single-block form, raw digest bytes
    b = blocks[0]
    assert miner.digest(b).hex() == golden["random_blocks"][0]["hex"]


def test_single_block_path(miner, golden, templates):
    """pow_hash_block (one block: K2', message by value, digest into mapped
    host memory) on every golden random block and edge-counter digest, one
    call each, against the reference's digests; and its call latency."""
    import statistics
    import time

    for e in golden["random_blocks"]:
        assert miner.block_to_hash(block_from_random(e)) == e["hex"]
    for e in golden["digests"]:
        b = with_nonce(block_from_template(templates[e["template"]]), nonce_from_counter(e["counter"]))
        assert miner.block_to_hash(b) == e["hex"]
    b = block_from_random(golden["random_blocks"][0])
    lat = []
    for _ in range(50):
        t = time.perf_counter()
        miner.block_to_hash(b)
        lat.append(time.perf_counter() - t)
    st = miner.stats()
    assert st["launches"] == 1 and st["hashes"] == 1 and 0 < st["kernel_ms"] < 1.0, st
    print(f"pow_hash_block: call median {statistics.median(lat) * 1e6:.1f} us, kernel {st['kernel_ms'] * 1e3:.1f} us")
    assert statistics.median(lat) < 0.001, lat


def test_launch_paths(miner, golden, templates):
    """The latency-bound launches (K2' here, K1' in pow_mine's first sub-round)
    go through hipLaunchKernel in the shipped library (round 5).  The test
    library's POW_AQL=1 sends them as AQL packets into the process's dispatch
    queue (pow_aql.cpp) instead.  Both give the reference's digests and the
    same lowest solution."""
    assert miner.launch_path() == "hip"
    direct = hooked_miner(POW_AQL=1)
    try:
        assert direct.launch_path() == "direct"
        for e in golden["random_blocks"]:
            b = block_from_random(e)
            assert direct.block_to_hash(b) == miner.block_to_hash(b) == e["hex"]
        w = golden["windows"][0]
        b = block_from_template(templates[w["template"]])
        for d, st in w["sets"].items():
            if st["count"]:
                want = w["start"] + st["counters"][0]
                assert miner.mine(b, w["start"], w["count"], int(d)).counter == want
                assert direct.mine(b, w["start"], w["count"], int(d)).counter == want
    finally:
        direct.close()


def test_messages(golden, templates):
    for name, hx in golden["messages"].items():
        b = with_nonce(block_from_template(templates[name]), nonce_from_counter(0))
        assert block_to_str(b).hex() == hx


@pytest.mark.parametrize("variant", ["fast", "full"])
def test_sweep_windows(miner, miner_full, golden, templates, variant):
    """Deterministic counter sweep: identical solution set for every golden window."""
    m = miner if variant == "fast" else miner_full
    for w in golden["windows"]:
        b = block_from_template(templates[w["template"]])
        for d, s in w["sets"].items():
            got = m.sweep(b, w["start"], w["count"], int(d))
            assert got.size == s["count"], (w["template"], w["start"], d)
            assert fp(got) == s["sha256_le_u32"], (w["template"], w["start"], d)
            if s["count"] <= 4096:
                assert got.tolist() == s["counters"]


def test_sweep_count_and_min(miner, golden, templates):
    for w in golden["windows"]:
        b = block_from_template(templates[w["template"]])
        for d, s in w["sets"].items():
            n, mn = miner.sweep_count(b, w["start"], w["count"], int(d))
            assert n == s["count"]
            first = s["counters"][0] + w["start"] if s["count"] else None
            assert mn == first


def test_mine_lowest_counter(mminer, golden, templates):
    """pow_mine returns the LOWEST solving counter and a block the reference
    would accept (nonce + strcpy'd hex, node.cpp:318)."""
    for w in golden["windows"]:
        b = block_from_template(templates[w["template"]])
        for d, s in w["sets"].items():
            r = mminer.mine(b, w["start"], w["count"], int(d))
            if s["count"] == 0:
                assert r is None
                continue
            assert r is not None
            assert r.counter == w["start"] + s["counters"][0]
            assert field(r.block, "nonce") == nonce_from_counter(r.counter)
            hx = block_hex(r.block)
            assert hx == mminer.block_to_hash(r.block)
            # the winner's digest (recorded by the latency kernel, or K2) vs standard SHA-256
            assert hx == hashlib.sha256(block_to_str(r.block)).hexdigest()
            assert field(r.block, "block_hash")[64] == 0
            assert field(r.block, "block_hash")[65:] == field(b, "block_hash")[65:]
            assert r.hashes >= r.counter - w["start"]


def test_mine_from_every_offset(mminer, golden, templates):
    """Start the search inside a prefix (off0 = 1..61) just before a known solution."""
    w = golden["windows"][0]  # S0 [0, 2^20)
    b = block_from_template(templates[w["template"]])
    sol = w["sets"]["9"]["counters"]
    for k in range(0, 40):
        target = sol[k]
        prev = sol[k - 1] + 1 if k else 0
        start = max(prev, target - (k % 62))
        r = mminer.mine(b, start, 4096, 9)
        assert r is not None and r.counter == target


def test_mine_any_returns_a_solution(mminer, golden, templates):
    """pow_mine_any: some solving counter of the range (a member of the golden
    set), None when the range holds none."""
    for w in golden["windows"]:
        b = block_from_template(templates[w["template"]])
        for d, s in w["sets"].items():
            r = mminer.mine(b, w["start"], w["count"], int(d), any_solution=True)
            if s["count"] == 0:
                assert r is None
                continue
            assert r is not None
            rel = r.counter - w["start"]
            assert 0 <= rel < w["count"]
            if s["count"] <= 4096:
                assert rel in set(s["counters"])
            hx = block_hex(r.block)
            assert hx == mminer.block_to_hash(r.block)
            assert hx == hashlib.sha256(block_to_str(r.block)).hexdigest()
            assert 256 - int(hx, 16).bit_length() >= int(d)


def test_latency_kernel_timing_and_stats(miner, templates):
    """The latency kernel times itself on the GPU (realtime counter from
    workgroup 0's start to the last workgroup's exit) and the host returns on
    its published `done` word: kernel_ms is positive and below the call's wall
    time, one launch per call at low d, and the trial count covers the winner."""
    import time

    b = block_from_template(templates["S0"])
    for d, want in ((9, 238), (13, None)):
        t = time.perf_counter()
        r = miner.mine(b, 0, 1 << 24, d)
        wall_ms = 1e3 * (time.perf_counter() - t)
        st = miner.stats()
        assert r is not None and (want is None or r.counter == want)
        assert 0 < st["kernel_ms"] < wall_ms, (st, wall_ms)
        assert st["launches"] >= 1 and st["hashes"] > r.counter, st
    # back-to-back calls: every launch publishes its own sequence number
    got = [miner.mine(b, 0, 1 << 16, 9).counter for _ in range(50)]
    assert got == [238] * 50


def test_mine_no_solution_and_bounds(miner, templates):
    b = block_from_template(templates["S0"])
    assert miner.mine(b, 0, 200, 9) is None  # first S0 solution is 238
    r = miner.mine(b, 0, 239, 9)
    assert r is not None and r.counter == 238
    with pytest.raises(PowError):
        miner.mine(b, COUNTER_LIMIT - 10, 11, 9)
    with pytest.raises(PowError):
        miner.sweep(b, 0, (1 << 32) + 1, 9)
    with pytest.raises(PowError):
        miner.mine(b, 0, 10, 257)


def test_difficulty_zero_and_enospc(miner, templates):
    b = block_from_template(templates["S1"])
    got = miner.sweep(b, 1000, 5000, 0, cap=5000)
    assert got.tolist() == list(range(5000))
    with pytest.raises(PowError) as ei:
        miner.sweep(b, 0, 5000, 0, cap=100)
    assert ei.value.code == -2


def test_cancel_epoch(miner, templates):
    b = block_from_template(templates["S2"])
    miner.cancel()  # epoch moves: a call with the stale epoch stops at once
    r = miner.mine(b, 0, 1 << 40, 60, epoch=(miner.epoch - 1) & 0xFFFFFFFF)
    assert r is None
    assert miner.stats()["launches"] == 0


@pytest.mark.parametrize("any_solution", [True, False])
def test_cancel_in_flight(any_solution):
    """pow_cancel from another thread stops a running mine call within one
    inner step: a search with no solution (d = 60) over 2^40 counters runs
    2^30-counter K1 launches of ~0.13 s; cancelled 30 ms in, it returns None
    within a few ms instead of at the end of its launch."""
    import threading
    import time

    b = block_from_template({"index": 5, "node_owner_number": 1, "difficulty": 9, "created_at": 1700000000,
                             "previous_block_hash_hex": "00" * 256})
    with GpuMiner(0) as m:
        m.cancel()  # arm the GPU-side check (first pow_cancel)
        ep = m.epoch
        assert m.mine(b, 0, 1 << 26, 60, epoch=ep, any_solution=any_solution) is None  # not cancelled: runs out
        res, t_end = {}, {}

        def run():
            res["r"] = m.mine(b, 0, 1 << 40, 60, epoch=ep, any_solution=any_solution)
            t_end["t"] = time.perf_counter()

        th = threading.Thread(target=run)
        th.start()
        time.sleep(0.03)
        t_cancel = time.perf_counter()
        m.cancel()
        th.join(timeout=30)
        assert not th.is_alive()
        assert res["r"] is None
        assert t_end["t"] - t_cancel < 0.02, t_end["t"] - t_cancel  # a 2^30 launch takes ~0.13 s


def test_validation_beside_mining():
    """Block validation (K2, another context and stream) while a K1 mining
    launch holds the GPU: K1 leaves one workgroup slot free, so a hash
    returns in well under a millisecond, not after the ~0.13 s launch."""
    import statistics
    import threading
    import time

    b = block_from_template({"index": 5, "node_owner_number": 1, "difficulty": 9, "created_at": 1700000000,
                             "previous_block_hash_hex": "00" * 256})
    with GpuMiner(0) as m, GpuMiner(0) as v:
        m.cancel()  # arm in-flight cancellation
        want = v.block_to_hash(b)
        th = threading.Thread(target=lambda: m.mine(b, 0, 1 << 40, 60, any_solution=True))
        th.start()
        time.sleep(0.05)
        lat = []
        for _ in range(20):
            t = time.perf_counter()
            assert v.block_to_hash(b) == want
            lat.append(time.perf_counter() - t)
        m.cancel()
        th.join(timeout=30)
        assert not th.is_alive()
        assert statistics.median(lat) < 0.005, lat


def test_direct_dispatch_two_threads(golden, templates):
    """Two contexts of one process driven from two threads at once, as in a
    pow_node rank (miner thread: pow_mine_any on K1', receive thread:
    pow_hash_block on K2'), both on direct dispatch (test library, POW_AQL=1):
    both put packets into the process's one dispatch queue (pow_aql.cpp, no
    barrier bit).  Every result must stay exact: the lowest solutions of the
    golden window and the reference's digests."""
    import threading

    w = golden["windows"][0]
    tmpl = block_from_template(templates[w["template"]])
    firsts = {int(d): w["start"] + st["counters"][0] for d, st in w["sets"].items() if st["count"]}
    blocks = [block_from_random(e) for e in golden["random_blocks"]]
    want = [e["hex"] for e in golden["random_blocks"]]
    errors = []
    with hooked_miner(POW_AQL=1) as m, hooked_miner(POW_AQL=1) as v:
        assert m.launch_path() == v.launch_path() == "direct"

        def mine_loop():
            try:
                for _ in range(60):
                    for d, first in firsts.items():
                        if d <= 13:
                            r = m.mine(tmpl, w["start"], w["count"], d)
                            if r is None or r.counter != first:
                                errors.append(("mine", d, r and r.counter, first))
            except Exception as e:  # pragma: no cover - reported below
                errors.append(("mine", repr(e)))

        th = threading.Thread(target=mine_loop)
        th.start()
        n = 0
        while th.is_alive() and n < 20000:
            for b, hx in zip(blocks, want):
                got = v.block_to_hash(b)
                if got != hx:
                    errors.append(("hash", got, hx))
                n += 1
        th.join(timeout=60)
        assert not th.is_alive()
    assert not errors, errors[:5]
    assert n >= len(blocks)


def _timed_hash(m, b, out, key):
    import time

    t = time.perf_counter()
    try:
        out[key] = (m.block_to_hash(b), time.perf_counter() - t)
    except Exception as e:  # reported by the caller
        out[key] = (e, time.perf_counter() - t)


def test_direct_dispatch_stalled_producer(golden):
    """The multi-producer ordering argument (pow_aql.cpp header),
    forced instead of left to timing.  Producer A (POW_AQL_EXP_STALL_HEADER)
    reserves packet index i, writes the body and then sleeps 200 ms before it
    stores the header and rings the doorbell with i.  Meanwhile producer B, on
    the same queue, takes i + 1, stores its header and rings the doorbell with
    i + 1 (a larger doorbell value first, then a smaller one).  Both launches
    must give the reference's digests; B's packet must not run before A's
    header is in (the packet processor does not process an INVALID slot, and
    takes packets in order), so B returns only after A's stall."""
    import threading
    import time

    blocks = [block_from_random(e) for e in golden["random_blocks"][:2]]
    want = [e["hex"] for e in golden["random_blocks"][:2]]
    a = hooked_miner(POW_AQL=1, POW_AQL_EXP=512, POW_AQL_STALL_US=200000)
    b = hooked_miner(POW_AQL=1)
    try:
        assert a.launch_path() == b.launch_path() == "direct"
        out = {}
        for rep in range(3):
            th = threading.Thread(target=_timed_hash, args=(a, blocks[0], out, "a"))
            th.start()
            time.sleep(0.05)  # A is inside its stall: index reserved, header not stored
            _timed_hash(b, blocks[1], out, "b")
            th.join(timeout=30)
            assert not th.is_alive()
            assert out["a"][0] == want[0] and out["b"][0] == want[1], out
            print(f"stalled producer, rep {rep}: A {out['a'][1] * 1e3:.1f} ms, B (behind A) {out['b'][1] * 1e3:.1f} ms")
            assert out["b"][1] > 0.1, out  # held behind A's INVALID slot until A's header went in
            # and unstalled, B alone is fast again
            t = time.perf_counter()
            assert b.block_to_hash(blocks[1]) == want[1]
            assert time.perf_counter() - t < 0.05
    finally:
        a.close()
        b.close()


def test_watchdog_direct_dispatch(golden):
    """A launch held in the queue past the watchdog's deadline is reported,
    not waited for: producer C (POW_WATCHDOG_MS=50) dispatches behind A's
    stalled slot (POW_AQL_EXP_STALL_HEADER, 400 ms).  C's call fails with
    POW_EHIP and the diagnostic (seq, done word, completion signal, the
    queue's read/write index, C's packet index and the header in its slot);
    the queue's read index has not reached C's packet.  A's launch and, once
    A's header is in, C's packet still complete: nothing is left wedged."""
    import re
    import threading
    import time

    from mpi_blockchain_amd._lib import PowError

    blocks = [block_from_random(e) for e in golden["random_blocks"][:2]]
    want = [e["hex"] for e in golden["random_blocks"][:2]]
    a = hooked_miner(POW_AQL=1, POW_AQL_EXP=512, POW_AQL_STALL_US=400000)
    c = hooked_miner(POW_AQL=1, POW_WATCHDOG_MS=50)
    try:
        out = {}
        th = threading.Thread(target=_timed_hash, args=(a, blocks[0], out, "a"))
        th.start()
        time.sleep(0.05)
        with pytest.raises(PowError) as ei:
            c.block_to_hash(blocks[1])
        msg = str(ei.value)
        print(msg)
        assert "hash kernel: watchdog: no result after" in msg and "launch path direct" in msg, msg
        m = re.search(r"read index (\d+), write index (\d+), this context's last packet index (\d+), "
                      r"header at its slot 0x([0-9a-f]+) \(type (\d+)", msg)
        assert m, msg
        rd, wr, idx, typ = int(m.group(1)), int(m.group(2)), int(m.group(3)), int(m.group(5))
        assert rd <= idx < wr and typ == 2, msg  # C's packet is valid and waits behind A's slot
        th.join(timeout=30)
        assert not th.is_alive() and out["a"][0] == want[0], out
    finally:
        a.close()
        c.close()  # waits (bounded) for C's packet, which runs once A's header is in


@pytest.mark.parametrize("what", ["hash_one", "latency", "search"])
def test_watchdog_hip_path(golden, templates, what):
    """The same watchdog on the HIP launch path (the shipped one): the test
    library's POW_TEST_STALL_US puts a bounded 300 ms stall kernel in front
    of each launch on the context's stream, and POW_WATCHDOG_MS=30 makes the
    host's wait give up first.  K2' (pow_hash_block), K1' (first sub-round of
    pow_mine) and K1 (pow_sweep) each fail with POW_EHIP and a watchdog
    diagnostic instead of waiting."""
    from mpi_blockchain_amd._lib import PowError

    m = hooked_miner(POW_TEST_STALL_US=300000, POW_WATCHDOG_MS=30)
    try:
        assert m.launch_path() == "hip"
        b = block_from_random(golden["random_blocks"][0])
        tmpl = block_from_template(templates["S0"])
        with pytest.raises(PowError) as ei:
            if what == "hash_one":
                m.block_to_hash(b)
            elif what == "latency":
                m.mine(tmpl, 0, 1 << 20, 9)
            else:
                m.sweep(tmpl, 0, 1 << 20, 9)
        msg = str(ei.value)
        print(msg)
        key = {"hash_one": "hash kernel: watchdog: no result after",
               "latency": "latency kernel: watchdog: no result after",
               "search": "watchdog: not complete after"}[what]
        assert key in msg, msg
        assert "launch path hip" in msg or what == "search", msg
    finally:
        m.close()  # synchronises the stream: the stall kernel ends on its own


def test_chained_blocks_validate(miner):
    """Mine three chained blocks with the GPU and check the chain the way the
    receive side does (valid_new_block, block.cpp:13-25: recomputed hash ==
    stored hash; prev == previous block_hash)."""
    from mpi_blockchain_amd.block import make_block, solves_problem

    last = make_block(0, 0, 9, 1700000000)  # genesis: block_hash zeroed (node.cpp:369)
    chain = [last]
    for k in range(3):
        t = refresh_template(chain[-1], rank=k, difficulty=9, now=1700000000 + k)
        r = miner.mine(t, 0, 1 << 30, 9)
        assert r is not None
        hx = block_hex(r.block)
        assert solves_problem(hx, 9)
        assert miner.block_to_hash(r.block) == hx
        assert field(r.block, "previous_block_hash") == field(chain[-1], "block_hash")
        chain.append(r.block)
    assert [c.index for c in chain] == [0, 1, 2, 3]


@pytest.mark.slow
def test_full_window_2p32(miner, fingerprints, templates):
    """BASELINE config 2 at full size: S0, counters [0, 2^32), d = 9..25 —
    count and sha256 of the sorted solution list equal the CPU fingerprints."""
    b = block_from_template(templates["S0"])
    got = miner.sweep(b, 0, 1 << 32, 9, cap=9_000_000)
    lad = fingerprints["ladder"]
    assert got.size == lad["9"]["count"]
    assert fp(got) == lad["9"]["sha256_le_u32"]
    for d in ("13", "17", "21", "25"):
        n, mn = miner.sweep_count(b, 0, 1 << 32, int(d))
        assert n == lad[d]["count"]
        assert mn == lad[d]["first"][0]


@pytest.mark.parametrize("nranks", [3, 8])
def test_shard_union_equals_full_window(miner, fingerprints, templates, nranks):
    """SURVEY.md §4 item 4 at full size: the static shards of [0, 2^32)
    (pow_group_partition, unaligned for 3 ranks), each swept on its own as a
    rank of config 4 would, unite to exactly the single window's solution set
    (count + sha256 of the sorted list = the CPU fingerprints), and the lowest
    counter over the shards is the window's first solution."""
    import numpy as np

    from mpi_blockchain_amd.shard import native_partition

    b = block_from_template(templates["S0"])
    parts, lows = [], []
    for r in range(nranks):
        s, k = native_partition(0, 1 << 32, r, nranks)
        got = miner.sweep(b, s, k, 9, cap=9_000_000 // nranks + 100_000)
        parts.append(got.astype(np.uint64) + s)
        if got.size:
            lows.append(int(got[0]) + s)
    union = np.sort(np.concatenate(parts)).astype(np.uint32)
    lad = fingerprints["ladder"]["9"]
    assert union.size == lad["count"]
    assert fp(union) == lad["sha256_le_u32"]
    assert min(lows) == lad["first"][0]


@pytest.mark.parametrize("name", ["S1", "S2"])
def test_full_window_2p32_S1(miner, templates, name):
    """Config 2 at full size on the other golden templates:
    S1, the realistic chained template (index 7, owner 3, prev = a 64-char hex
    hash + NUL + zeros), and S2 (every header field truncated to its low byte,
    prev = 64 x 'Z' + NUL + 191 x 'Z': non-zero bytes in every chunk-1..4 word).
    Counts and sha256 of the sorted solution list at every rung vs the CPU
    restatement's fingerprints (tests/golden/fingerprints_2p32_<name>.json)."""
    import json

    path = os.path.join(os.path.dirname(__file__), "golden", f"fingerprints_2p32_{name}.json")
    if not os.path.exists(path):
        pytest.skip(f"{name} fingerprints not generated")
    fps = json.load(open(path))
    b = block_from_template(templates[name])
    lad = fps["ladder"]
    got = miner.sweep(b, 0, 1 << 32, 9, cap=9_000_000)
    assert got.size == lad["9"]["count"] and fp(got) == lad["9"]["sha256_le_u32"]
    for d in ("13", "17", "21", "25"):
        sol = miner.sweep(b, 0, 1 << 32, int(d), cap=lad[d]["count"] + 16)
        assert sol.size == lad[d]["count"] and fp(sol) == lad[d]["sha256_le_u32"], d


@pytest.mark.parametrize("r", range(1, 8))
def test_full_window_2p32_far(miner, templates, r):
    """S0 over [r*2^32, (r+1)*2^32), r = 1..7: the window rank r sweeps in
    bench.py's N-GPU runs (for r = 7, nonce[3] = 'G'..'L' instead of 'a'..'e';
    counters past 2^32 in the launch base).  Counts, sha256 of the sorted list
    (relative counters) and lowest counter at every rung vs the CPU
    restatement (tests/golden/gen_fingerprints_2p32.py; reference's rule
    block.cpp:91-96)."""
    import json

    start = r << 32
    path = os.path.join(os.path.dirname(__file__), "golden", f"fingerprints_2p32_S0_at{start}.json")
    if not os.path.exists(path):
        pytest.skip(f"window {r} fingerprints not generated")
    fps = json.load(open(path))
    assert fps["start"] == start and fps["template"] == "S0" and fps["count"] == 1 << 32
    b = block_from_template(templates["S0"])
    lad = fps["ladder"]
    got = miner.sweep(b, start, 1 << 32, 9, cap=9_000_000)
    assert got.size == lad["9"]["count"] and fp(got) == lad["9"]["sha256_le_u32"]
    for d in ("13", "17", "21", "25"):
        n, mn = miner.sweep_count(b, start, 1 << 32, int(d))
        assert n == lad[d]["count"] and mn == start + lad[d]["first"][0], d


def test_mine_full_window_ladder(mminer, fingerprints, templates):
    """pow_mine over S0's [0, 2^32) at every rung (K1' for d <= 21, K1 sub-rounds
    above): the lowest solving counter, then each next one when the search
    starts just past the previous, equal the CPU fingerprints' first counters;
    pow_mine_any returns a valid solution of the window.  Winner hashes vs
    standard SHA-256."""
    b = block_from_template(templates["S0"])
    for d, lad in fingerprints["ladder"].items():
        start = 0
        for want in lad["first"][:3]:
            r = mminer.mine(b, start, (1 << 32) - start, int(d))
            assert r is not None and r.counter == want
            assert block_hex(r.block) == hashlib.sha256(block_to_str(r.block)).hexdigest()
            start = want + 1
        r = mminer.mine(b, 0, 1 << 32, int(d), any_solution=True)
        assert r is not None and 0 <= r.counter < 1 << 32
        hx = block_hex(r.block)
        assert hx == hashlib.sha256(block_to_str(r.block)).hexdigest()
        assert 256 - int(hx, 16).bit_length() >= int(d)


def test_random_templates_vs_oracle(miner):
    """Fresh random templates (arbitrary header fields, binary or hex-string
    prev hashes, random window starts): GPU sweep == C-oracle sweep."""
    import random

    from mpi_blockchain_amd.block import make_block
    from oracle.oracle import Oracle, make_oblock

    O = Oracle()
    rng = random.Random(424242)
    threads = min(16, len(os.sched_getaffinity(0)))
    for k in range(12):
        idx, own, dif, cat = (rng.randrange(1 << 32), rng.randrange(1 << 32), rng.randrange(1 << 32),
                              rng.randrange(1 << 64))
        if k % 2:
            prev = bytes(rng.randrange(256) for _ in range(256))
        else:
            prev = hashlib.sha256(bytes([k])).hexdigest().encode()
        start = rng.randrange(62**9 - (1 << 20))
        count = rng.randrange(1 << 16, 1 << 18)
        d = rng.choice([6, 8, 10])
        got = miner.sweep(make_block(idx, own, dif, cat, prev), start, count, d)
        want, n = O.sweep(make_oblock(idx, own, dif, cat, prev), start, count, d, cap=count, threads=threads)
        assert got.tolist() == want.tolist(), (k, start, count, d)


def test_parity_fuzz():
    """Randomised parity (tests/parity_fuzz.py): 120 random templates, window
    starts (anywhere, straddling 2^32 multiples and base-62 carries, the end
    of the counter space), lengths and difficulties 0..14: pow_sweep's list ==
    the oracle's, pow_mine == its first, pow_mine_any in it, and the winner's
    digest == the oracle's, the reference's (oracle/_ref) and K2''s."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import parity_fuzz

    with GpuMiner(0) as m:
        res = parity_fuzz.run(120, 2024, miner=m)
    assert res.get("ok"), res
    assert res["cases"] == 120 and res["solutions"] > 0


@pytest.mark.parametrize("env", [{"POW_LAT_WPS": 4}, {"POW_LAT_WPS": 4, "POW_FORCE_FULL": 1}, {"POW_AQL": 1}],
                         ids=["lat_asm", "lat_asm_full", "direct_dispatch"])
def test_parity_fuzz_latency_asm_variants(env):
    """The latency kernel's asm-group variants (pow_search_lat<*, *, true>, run
    by the plan only at d = 20-21, 4 waves per SIMD) under the same exact
    oracle comparison: the test library forces 4 waves per SIMD at every d,
    and with POW_FORCE_FULL the d > 32 variants <true, *, true> as well.
    direct_dispatch: the plan's kernels sent as AQL packets (test library,
    POW_AQL=1) instead of the shipped hipLaunchKernel."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import parity_fuzz

    m = hooked_miner(**env)
    try:
        res = parity_fuzz.run(40, 4040 + len(env), miner=m)
    finally:
        m.close()
    assert res.get("ok"), res
    assert res["cases"] == 40 and res["solutions"] > 0


def test_sweep_d0_full_window_count():
    """At difficulty 0 every counter solves: a full 2^32 window has exactly
    2^32 solutions, which the 64-bit solution count (PowResult::count) holds
    (a 32-bit one wrapped to 0 here).  Count-only form, no list."""
    with GpuMiner(0) as m:
        b = make_block(1, 0, 9, 1700000000, b"")
        n, mn = m.sweep_count(b, 0, 1 << 32, 0)
        assert n == 1 << 32 and mn == 0
        n, mn = m.sweep_count(b, 1000, (1 << 32) - 5, 0)
        assert n == (1 << 32) - 5 and mn == 1000
