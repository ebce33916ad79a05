"""The oracle, pinned: the C restatement (oracle/pow_oracle.c) and the Python
restatements reproduce the golden vectors, which were generated from the
reference's own block.cpp + picosha2.h (tests/golden/gen_golden.py).  CPU only."""
import ctypes
import hashlib
import random

import numpy as np
import pytest

from oracle.oracle import (OBlock, Oracle, RefLib, make_oblock, py_block_to_str, py_nonce_from_counter,
                           py_solves_problem, ref_available)


@pytest.fixture(scope="module")
def O():
    return Oracle()


def oblock(t) -> OBlock:
    return make_oblock(t["index"], t["node_owner_number"], t["difficulty"], t["created_at"],
                       bytes.fromhex(t["previous_block_hash_hex"]))


def set_nonce(b, n):
    ctypes.memmove(ctypes.addressof(b) + OBlock.nonce.offset, n, 10)


def test_sizeof_block(O):
    assert ctypes.sizeof(OBlock) == 552
    assert OBlock.created_at.offset == 16 and OBlock.nonce.offset == 24
    assert OBlock.previous_block_hash.offset == 34 and OBlock.block_hash.offset == 290


def test_nonce_mapping(O, golden):
    for e in golden["digests"]:
        n = py_nonce_from_counter(e["counter"])
        assert n[:9].decode() == e["nonce"] and n[9] == 0
        assert O.nonce_from_counter(e["counter"]) == n
    assert py_nonce_from_counter(0) == b"aaaaaaaaa\0"
    assert py_nonce_from_counter(62**9 - 1) == b"999999999\0"
    with pytest.raises(ValueError):
        O.nonce_from_counter(62**9)


def test_messages(O, golden, templates):
    for name, hx in golden["messages"].items():
        t = templates[name]
        b = oblock(t)
        set_nonce(b, py_nonce_from_counter(0))
        assert O.block_to_str(b).hex() == hx
        py = py_block_to_str(t["index"], t["node_owner_number"], t["difficulty"], t["created_at"],
                             py_nonce_from_counter(0), bytes.fromhex(t["previous_block_hash_hex"]))
        assert py.hex() == hx and len(py) == 270


def test_edge_digests(O, golden, templates):
    for e in golden["digests"]:
        b = oblock(templates[e["template"]])
        set_nonce(b, py_nonce_from_counter(e["counter"]))
        dg, hx = O.block_to_hash(b)
        assert hx == e["hex"] and dg.hex() == e["hex"]
        assert py_solves_problem(hx, 9) == e["solves_d9"] == O.solves_problem(hx, 9)


def test_random_block_digests(O, golden):
    for e in golden["random_blocks"]:
        b = make_oblock(e["index"], e["node_owner_number"], e["difficulty"], e["created_at"],
                        bytes.fromhex(e["previous_block_hash_hex"]), bytes.fromhex(e["nonce_hex"]))
        assert O.block_to_hash(b)[1] == e["hex"]
        assert hashlib.sha256(O.block_to_str(b)).hexdigest() == e["hex"]


def test_sha256_vs_hashlib(O):
    rng = random.Random(7)
    for n in list(range(0, 130)) + [270, 1000]:
        m = bytes(rng.randrange(256) for _ in range(n))
        assert O.sha256(m) == hashlib.sha256(m).digest()


def test_windows(O, golden, templates):
    for w in golden["windows"]:
        b = oblock(templates[w["template"]])
        for d, s in w["sets"].items():
            got, n = O.sweep(b, w["start"], w["count"], int(d), cap=w["count"])
            assert n == s["count"]
            assert hashlib.sha256(got.astype("<u4").tobytes()).hexdigest() == s["sha256_le_u32"]
            if s["count"]:
                assert O.mine(b, w["start"], w["count"], int(d)) == w["start"] + s["counters"][0]
            else:
                assert O.mine(b, w["start"], w["count"], int(d)) is None


def test_solves_problem_semantics(O):
    """block.cpp:28-58 + 91-96: toupper, non-hex -> "1111", compare(0, d, zeros)."""
    rng = random.Random(3)
    alphabet = "0123456789abcdefABCDEFxyz!"
    for _ in range(3000):
        h = "".join(rng.choice(alphabet) for _ in range(rng.randrange(0, 70)))
        d = rng.randrange(0, 300)
        assert O.solves_problem(h, d) == py_solves_problem(h, d), (h, d)
    assert py_solves_problem("00" + "f" * 62, 8) and not py_solves_problem("00" + "f" * 62, 9)
    assert py_solves_problem("007f", 9) and not py_solves_problem("0080", 9)
    assert py_solves_problem("", 0) and not py_solves_problem("0" * 64, 257)
    assert not py_solves_problem("0g", 8)  # 'g' is not hex: "1111"


@pytest.mark.skipif(not ref_available(), reason="oracle/_ref not built (needs /root/reference)")
def test_reference_build_agrees(O, templates):
    """The reference's own block_to_hash/solves_problem (oracle/_ref) vs the restatement."""
    R = RefLib("O2")
    rng = random.Random(11)
    for _ in range(200):
        t = templates[rng.choice(list(templates))]
        b = oblock(t)
        set_nonce(b, py_nonce_from_counter(rng.randrange(62**9)))
        assert R.block_to_str(b) == O.block_to_str(b)
        hx = R.block_to_hash(b)
        assert hx == O.block_to_hash(b)[1]
        assert R.solves_problem(hx) == O.solves_problem(hx, 9)
    got, n = R.sweep(oblock(templates["S2"]), 0, 1 << 14)
    ora, m = O.sweep(oblock(templates["S2"]), 0, 1 << 14, 9)
    assert n == m and np.array_equal(got, ora)


@pytest.mark.skipif(not ref_available(), reason="oracle/_ref not built")
def test_reference_random_nonce_alphabet():
    """gen_random_nonce (block.cpp:61-72): 9 chars of [a-zA-Z0-9] + NUL."""
    R = RefLib("O2")
    R.L.ref_srand(1)
    for _ in range(100):
        n = R.gen_random_nonce()
        assert n[9] == 0 and all(chr(c).isalnum() and c < 128 for c in n[:9])
