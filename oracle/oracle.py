"""ORACLE — TEST INFRASTRUCTURE ONLY.

Python handle on the CPU checkers.  Imported only by tests/, by
``__graft_entry__.smoke()`` and by bench.py's ``cpu_baseline`` leg — never by
the product package ``mpi_blockchain_amd`` (which must fail loudly rather than
fall back to anything here).

Three independent CPU views of the reference's hot path:

* ``Oracle``     — ``oracle/liboracle.so``: the plain-C restatement
                   (oracle/pow_oracle.c, cites block.cpp / picosha2.h lines).
* ``RefLib``     — ``oracle/_ref/libref_O2.so``: the reference's OWN
                   block.cpp + picosha2.h compiled in place (oracle/Makefile);
                   available only where it was built (this container, and the
                   GPU box when the built file travelled with the snapshot).
* ``py_*``       — pure Python/hashlib restatements for tiny cases, including
                   the literal hex -> binary-string test of block.cpp:91-96.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
HASH_SIZE = 256
NONCE_SIZE = 10
MSG_BYTES = 270
ALPHABET = (
    "abcdefghijklmnopqrstuvwxyz" "ABCDEFGHIJKLMNOPQRSTUVWXYZ" "0123456789"
)  # block.cpp:61-72 order: rand()%62 -> a-z, A-Z, 0-9


class OBlock(ctypes.Structure):
    """block.h:17-25 on LP64 (sizeof 552)."""

    _fields_ = [
        ("index", ctypes.c_uint32),
        ("node_owner_number", ctypes.c_uint32),
        ("difficulty", ctypes.c_uint32),
        ("created_at", ctypes.c_uint64),
        ("nonce", ctypes.c_char * NONCE_SIZE),
        ("previous_block_hash", ctypes.c_char * HASH_SIZE),
        ("block_hash", ctypes.c_char * HASH_SIZE),
    ]


def make_oblock(index, owner, difficulty, created_at, prev: bytes, nonce: bytes = b"") -> OBlock:
    b = OBlock()
    b.index = index & 0xFFFFFFFF
    b.node_owner_number = owner & 0xFFFFFFFF
    b.difficulty = difficulty & 0xFFFFFFFF
    b.created_at = created_at & 0xFFFFFFFFFFFFFFFF
    prev = bytes(prev).ljust(HASH_SIZE, b"\0")[:HASH_SIZE]
    ctypes.memmove(ctypes.addressof(b) + OBlock.previous_block_hash.offset, prev, HASH_SIZE)
    nz = bytes(nonce).ljust(NONCE_SIZE, b"\0")[:NONCE_SIZE]
    ctypes.memmove(ctypes.addressof(b) + OBlock.nonce.offset, nz, NONCE_SIZE)
    return b


def raw_field(b: OBlock, name: str) -> bytes:
    f = getattr(OBlock, name)
    return ctypes.string_at(ctypes.addressof(b) + f.offset, f.size)


# --------------------------------------------------------------------------
# pure-Python restatement (small cases only)
# --------------------------------------------------------------------------
def py_nonce_from_counter(c: int) -> bytes:
    """Counter -> 9 base-62 chars MSB first + NUL (alphabet of block.cpp:61-72)."""
    if not 0 <= c < 62**9:
        raise ValueError("counter out of range")
    out = []
    for _ in range(NONCE_SIZE - 1):
        out.append(ALPHABET[c % 62])
        c //= 62
    return "".join(reversed(out)).encode() + b"\0"


def py_block_to_str(index, owner, difficulty, created_at, nonce10: bytes, prev256: bytes) -> bytes:
    """block.cpp:79-88: one byte per integer field (T1), nonce incl. NUL, all
    256 prev bytes (T2)."""
    assert len(nonce10) == NONCE_SIZE and len(prev256) == HASH_SIZE
    return bytes([index & 255, owner & 255, difficulty & 255, created_at & 255]) + nonce10 + prev256


def py_hex_char_to_bin(c: str) -> str:
    """block.cpp:28-49 (toupper; default "1111")."""
    table = {"0": "0000", "1": "0001", "2": "0010", "3": "0011", "4": "0100", "5": "0101",
             "6": "0110", "7": "0111", "8": "1000", "9": "1001", "A": "1010", "B": "1011",
             "C": "1100", "D": "1101", "E": "1110"}
    return table.get(c.upper(), "1111")


def py_solves_problem(hex_digest: str, d: int) -> bool:
    """block.cpp:91-96 literally: binary string, compare(0, d, "0"*d)."""
    binary = "".join(py_hex_char_to_bin(c) for c in hex_digest)
    return binary[:d] == "0" * d


def py_block_hash(msg: bytes) -> str:
    return hashlib.sha256(msg).hexdigest()


# --------------------------------------------------------------------------
# C restatement
# --------------------------------------------------------------------------
def _build_oracle() -> None:
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)


class Oracle:
    def __init__(self, path: str | None = None):
        path = path or os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            _build_oracle()
        L = ctypes.CDLL(path)
        P = ctypes.POINTER(OBlock)
        L.oracle_sizeof_block.restype = ctypes.c_uint
        L.oracle_block_to_hash.argtypes = [P, ctypes.c_char_p, ctypes.c_char_p]
        L.oracle_block_to_str.argtypes = [P, ctypes.c_char_p]
        L.oracle_block_to_str.restype = ctypes.c_size_t
        L.oracle_nonce_from_counter.argtypes = [ctypes.c_uint64, ctypes.c_char_p]
        L.oracle_solves_problem.argtypes = [ctypes.c_char_p, ctypes.c_uint]
        L.oracle_sweep.argtypes = [P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint,
                                   ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t, ctypes.c_int]
        L.oracle_sweep.restype = ctypes.c_size_t
        L.oracle_mine.argtypes = [P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint]
        L.oracle_mine.restype = ctypes.c_uint64
        L.oracle_bench.argtypes = [P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint]
        L.oracle_bench.restype = ctypes.c_uint64
        L.oracle_sha256.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
        self.L = L
        assert L.oracle_sizeof_block() == ctypes.sizeof(OBlock) == 552

    def sha256(self, msg: bytes) -> bytes:
        out = ctypes.create_string_buffer(32)
        self.L.oracle_sha256(msg, len(msg), out)
        return out.raw

    def block_to_str(self, b: OBlock) -> bytes:
        out = ctypes.create_string_buffer(MSG_BYTES)
        n = self.L.oracle_block_to_str(ctypes.byref(b), out)
        return out.raw[:n]

    def block_to_hash(self, b: OBlock) -> tuple[bytes, str]:
        dg = ctypes.create_string_buffer(32)
        hx = ctypes.create_string_buffer(65)
        self.L.oracle_block_to_hash(ctypes.byref(b), dg, hx)
        return dg.raw, hx.value.decode()

    def nonce_from_counter(self, c: int) -> bytes:
        out = ctypes.create_string_buffer(NONCE_SIZE)
        if self.L.oracle_nonce_from_counter(c, out) != 0:
            raise ValueError("counter out of range")
        return out.raw

    def solves_problem(self, hex_digest: str, d: int) -> bool:
        return bool(self.L.oracle_solves_problem(hex_digest.encode(), d))

    def sweep(self, b: OBlock, start: int, count: int, d: int, cap: int | None = None,
              threads: int | None = None):
        """Ascending list of (counter - start) of solving counters; count."""
        import numpy as np

        if cap is None:
            cap = max(1024, (count >> max(d, 0)) * 4 + 1024) if d < 64 else 1024
        threads = threads or min(8, os.cpu_count() or 1)
        out = np.zeros(cap, dtype=np.uint32)
        n = self.L.oracle_sweep(ctypes.byref(b), start, count, d,
                                out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), cap, threads)
        return out[: min(n, cap)].copy(), int(n)

    def mine(self, b: OBlock, start: int, count: int, d: int):
        r = self.L.oracle_mine(ctypes.byref(b), start, count, d)
        return None if r == 0xFFFFFFFFFFFFFFFF else int(r)

    def bench(self, b: OBlock, start: int, n: int, d: int) -> int:
        return int(self.L.oracle_bench(ctypes.byref(b), start, n, d))


# --------------------------------------------------------------------------
# the reference itself (compiled from /root/reference by oracle/Makefile)
# --------------------------------------------------------------------------
REF_DIR = os.path.join(HERE, "_ref")


def ref_available(flavour: str = "O2") -> bool:
    return os.path.exists(os.path.join(REF_DIR, f"libref_{flavour}.so"))


class RefLib:
    def __init__(self, flavour: str = "O2"):
        path = os.path.join(REF_DIR, f"libref_{flavour}.so")
        if not os.path.exists(path):
            raise FileNotFoundError(path + " (build with `make -C oracle ref` where /root/reference exists)")
        L = ctypes.CDLL(path)
        P = ctypes.POINTER(OBlock)
        L.ref_sizeof_block.restype = ctypes.c_uint
        L.ref_default_difficulty.restype = ctypes.c_uint
        L.ref_block_to_str.argtypes = [P, ctypes.c_char_p, ctypes.c_int]
        L.ref_block_to_hash.argtypes = [P, ctypes.c_char_p]
        L.ref_solves_problem.argtypes = [ctypes.c_char_p]
        L.ref_gen_random_nonce.argtypes = [ctypes.c_char_p]
        L.ref_srand.argtypes = [ctypes.c_uint]
        L.ref_sweep.argtypes = [P, ctypes.c_uint64, ctypes.c_uint64,
                                ctypes.POINTER(ctypes.c_uint32), ctypes.c_long]
        L.ref_sweep.restype = ctypes.c_long
        L.ref_mine_loop.argtypes = [P, ctypes.c_int, ctypes.c_uint64]
        L.ref_mine_loop.restype = ctypes.c_uint64
        self.L = L
        assert L.ref_sizeof_block() == 552
        self.default_difficulty = int(L.ref_default_difficulty())

    def block_to_str(self, b: OBlock) -> bytes:
        out = ctypes.create_string_buffer(1024)
        n = self.L.ref_block_to_str(ctypes.byref(b), out, 1024)
        return out.raw[:n]

    def block_to_hash(self, b: OBlock) -> str:
        out = ctypes.create_string_buffer(65)
        assert self.L.ref_block_to_hash(ctypes.byref(b), out) == 64
        return out.value.decode()

    def solves_problem(self, hex_digest: str) -> bool:
        return bool(self.L.ref_solves_problem(hex_digest.encode()))

    def gen_random_nonce(self) -> bytes:
        out = ctypes.create_string_buffer(NONCE_SIZE)
        self.L.ref_gen_random_nonce(out)
        return out.raw

    def sweep(self, b: OBlock, start: int, count: int, cap: int = 1 << 20):
        import numpy as np

        out = np.zeros(cap, dtype=np.uint32)
        n = self.L.ref_sweep(ctypes.byref(b), start, count,
                             out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), cap)
        return out[: min(n, cap)].copy(), int(n)
