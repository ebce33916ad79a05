"""Generate tests/golden/golden.json — the parity vectors for the hot path.

Every expected value here comes from the REFERENCE ITSELF: /root/reference's
block.cpp + picosha2.h compiled unmodified into oracle/_ref/libref_O2.so
(``make -C oracle ref``) and driven through oracle/ref_shim.cpp —
block_to_str (block.cpp:79-88), block_to_hash (block.cpp:74-77) and
solves_problem (block.cpp:91-96, DEFAULT_DIFFICULTY = 9).  Python hashlib is a
second, independent check of every digest.  Solution sets at difficulties other
than 9 (the reference's difficulty is a compile-time macro, block.h:6) are
derived from reference digests with the bit test, cross-checked against the
literal hex->binary-string test restated in oracle/oracle.py.

    python tests/golden/gen_golden.py          # needs /root/reference (this container)
"""
from __future__ import annotations

import ctypes
import hashlib
import json
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle.oracle import (OBlock, Oracle, RefLib, make_oblock, py_nonce_from_counter,  # noqa: E402
                           py_solves_problem, raw_field)


def tmpl_dict(name, index, owner, difficulty, created_at, prev: bytes):
    return {"name": name, "index": index, "node_owner_number": owner, "difficulty": difficulty,
            "created_at": created_at, "previous_block_hash_hex": prev.ljust(256, b"\0").hex()}


TEMPLATES = [
    # S0: first block after genesis (prev = genesis block_hash, memset 0: node.cpp:369)
    tmpl_dict("S0", 1, 0, 9, 1700000000, b""),
    # S1: realistic chained block: prev = 64 hex chars + NUL + 191 zeros (strcpy, node.cpp:318)
    tmpl_dict("S1", 7, 3, 9, 1760572800,
              b"007384e324711d0c9fab8d3ed9b7be265575e29bde9a9ea56b1d86672ee927e8"),
    # S2: every integer field truncated to its low byte (T1) and a non-zero prev tail (T5)
    tmpl_dict("S2", 300, 7, 9, 0x1000000FF, b"Z" * 64 + b"\0" + b"Z" * 191),
    # S3: 0x80-heavy header and binary prev bytes
    tmpl_dict("S3", 0xDEADBE80, 0xFFFFFFFF, 0x1FF, 0xFFFFFFFFFFFFFFFF, bytes(range(256))),
]


def to_oblock(t) -> OBlock:
    return make_oblock(t["index"], t["node_owner_number"], t["difficulty"], t["created_at"],
                       bytes.fromhex(t["previous_block_hash_hex"]))


def set_nonce(b: OBlock, nonce10: bytes) -> None:
    ctypes.memmove(ctypes.addressof(b) + OBlock.nonce.offset, nonce10, 10)


def lz_bits(hexd: str) -> int:
    v = int(hexd, 16)
    return 256 - v.bit_length()


EDGE_COUNTERS = [0, 1, 2, 25, 26, 51, 52, 61, 62, 63, 3843, 3844, 238327, 238328, 62**5 - 1, 62**5,
                 2**32 - 1, 2**32, 62**6 - 1, 62**6, 62**7 + 12345, 62**8 - 1, 62**8, 62**9 - 1]

WINDOWS = [  # (template, start, count, difficulties) — reference d=9 sweep for each
    ("S0", 0, 1 << 20, [9, 13, 17, 21]),
    ("S1", 0, 1 << 20, [9, 13, 17]),
    ("S2", 0, 1 << 16, [9, 13]),
    ("S3", 0, 1 << 16, [9]),
    ("S1", 62**5 - (1 << 18), 1 << 19, [9, 13]),   # crosses a W1 (nonce[3]) carry
    ("S0", 123457, 200003, [9, 13]),               # start and end not multiples of 62
    ("S2", 2**32 - 5000, 10000, [5, 9]),           # straddles 2^32
    ("S0", 62**9 - 20000, 20000, [9]),             # last counters of the space
]


def main():
    R = RefLib("O2")
    O = Oracle()
    assert R.default_difficulty == 9
    out = {"generator": "tests/golden/gen_golden.py", "reference": "oracle/_ref/libref_O2.so "
           "(/root/reference block.cpp + picosha2.h)", "templates": TEMPLATES, "messages": {},
           "digests": [], "random_blocks": [], "windows": []}
    tm = {t["name"]: t for t in TEMPLATES}

    # 1. exact messages and digests at edge counters
    for t in TEMPLATES:
        b = to_oblock(t)
        for c in EDGE_COUNTERS:
            n = py_nonce_from_counter(c)
            assert O.nonce_from_counter(c) == n
            set_nonce(b, n)
            msg = R.block_to_str(b)
            assert len(msg) == 270 and msg == O.block_to_str(b)
            hx = R.block_to_hash(b)
            assert hx == hashlib.sha256(msg).hexdigest() == O.block_to_hash(b)[1]
            assert R.solves_problem(hx) == py_solves_problem(hx, 9) == (lz_bits(hx) >= 9)
            if c == 0:
                out["messages"][t["name"]] = msg.hex()
            out["digests"].append({"template": t["name"], "counter": c, "nonce": n[:9].decode(),
                                   "hex": hx, "solves_d9": R.solves_problem(hx)})

    # 2. random whole blocks (K2 / block_to_hash parity): arbitrary nonce bytes too
    rng = random.Random(20191201)
    for i in range(48):
        prev = bytes(rng.randrange(256) for _ in range(256))
        if i % 3 == 0:  # realistic: hex + NUL + zeros
            prev = hashlib.sha256(prev).hexdigest().encode() + b"\0" * 192
        b = make_oblock(rng.randrange(1 << 32), rng.randrange(1 << 32), rng.randrange(1 << 32),
                        rng.randrange(1 << 64), prev,
                        bytes(rng.randrange(256) for _ in range(10)))
        hx = R.block_to_hash(b)
        assert hx == hashlib.sha256(R.block_to_str(b)).hexdigest()
        out["random_blocks"].append({"index": b.index, "node_owner_number": b.node_owner_number,
                                     "difficulty": b.difficulty, "created_at": b.created_at,
                                     "nonce_hex": raw_field(b, "nonce").hex(),
                                     "previous_block_hash_hex": raw_field(b, "previous_block_hash").hex(),
                                     "hex": hx})

    # 3. solution sets over counter windows
    for name, start, count, ds in WINDOWS:
        b = to_oblock(tm[name])
        ref9, n9 = R.sweep(b, start, count, cap=count)          # reference, d = 9
        sol9 = ref9[:n9]
        ora9, m9 = O.sweep(b, start, count, 9, cap=count)
        assert m9 == n9 and np.array_equal(ora9, sol9), (name, start)
        entry = {"template": name, "start": start, "count": count, "sets": {}}
        for d in ds:
            ora, m = O.sweep(b, start, count, d, cap=count)
            if d >= 9:  # subset of the reference's d=9 set, by the literal string test
                sub = []
                for rel in sol9:
                    set_nonce(b, py_nonce_from_counter(start + int(rel)))
                    if py_solves_problem(R.block_to_hash(b), d):
                        sub.append(int(rel))
                assert sub == [int(x) for x in ora], (name, start, d)
            vals = [int(x) for x in ora[:m]]
            entry["sets"][str(d)] = {
                "count": m, "sha256_le_u32": hashlib.sha256(np.asarray(vals, "<u4").tobytes()).hexdigest(),
                "counters": vals if m <= 4096 else vals[:64]}
        out["windows"].append(entry)
        print(name, start, count, {d: entry["sets"][d]["count"] for d in entry["sets"]}, flush=True)

    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=0, separators=(",", ":"))
        f.write("\n")


if __name__ == "__main__":
    main()
