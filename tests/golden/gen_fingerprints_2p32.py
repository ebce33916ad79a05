"""Generate the full-window fingerprints of tests/golden/fingerprints_2p32.json.

Template S0 (index=1, owner=0, difficulty=9, created_at=1700000000, prev = 256
zero bytes), counters [0, 2^32), difficulty ladder d = 9, 13, 17, 21, 25 bits.
Fingerprint = sha256 of the ascending solving counters as little-endian u32.

Computed with the C restatement (oracle/liboracle.so, itself pinned against the
reference's own block_to_hash/solves_problem on the 2^20 windows of
golden.json) in one pass at d=9, recording each solution's leading-zero-bit
count; the higher rungs are the subsets with lz >= d.  Cross-checked against the
independent hashlib computation recorded in SURVEY.md §8c (same counts and
hashes).  Runtime: ~20 min on 8 cores.

    python tests/golden/gen_fingerprints_2p32.py [threads] [S0|S1] [start]

S1 (the realistic chained template of SURVEY.md §8c: index=7, owner=3,
difficulty=9, created_at=1760572800, prev = a 64-char hex hash + NUL + zeros)
goes to fingerprints_2p32_S1.json; S2 (truncated header fields, prev = 64 x 'Z' +
NUL + 191 x 'Z') to fingerprints_2p32_S2.json.  A non-zero start (e.g. 7 * 2^32: the window
rank 7 sweeps in bench.py's 8-GPU run) goes to
fingerprints_2p32_<template>_at<start>.json; counters in it are relative to start.
"""
import ctypes, hashlib, json, os, sys, time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle.oracle import OBlock, Oracle, make_oblock  # noqa: E402

threads = int(sys.argv[1]) if len(sys.argv) > 1 else 8
which = sys.argv[2] if len(sys.argv) > 2 else "S0"
start = int(sys.argv[3]) if len(sys.argv) > 3 else 0
O = Oracle()
L = O.L
L.oracle_sweep_lz.argtypes = [ctypes.POINTER(OBlock), ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint,
                              ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint8),
                              ctypes.c_size_t, ctypes.c_int]
L.oracle_sweep_lz.restype = ctypes.c_size_t
TEMPLATES = {"S0": make_oblock(1, 0, 9, 1700000000, b""),
             "S1": make_oblock(7, 3, 9, 1760572800,
                               b"007384e324711d0c9fab8d3ed9b7be265575e29bde9a9ea56b1d86672ee927e8"),
             # S2: every header field truncated to its low byte, non-zero prev tail
             "S2": make_oblock(300, 7, 9, 0x1000000FF, b"Z" * 64 + b"\0" + b"Z" * 191)}
S0 = TEMPLATES[which]
cap = 9_000_000
ctr = np.zeros(cap, np.uint32)
lz = np.zeros(cap, np.uint8)
t = time.time()
n = L.oracle_sweep_lz(ctypes.byref(S0), start, 1 << 32, 9, ctr.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                      lz.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), cap, threads)
assert n <= cap
ctr, lz = ctr[:n], lz[:n]
out = {"template": which, "start": start, "count": 1 << 32, "seconds": round(time.time() - t, 1), "ladder": {}}
for d in (9, 13, 17, 21, 25):
    sel = ctr[lz >= d]
    out["ladder"][str(d)] = {"count": int(sel.size),
                             "sha256_le_u32": hashlib.sha256(sel.astype("<u4").tobytes()).hexdigest(),
                             "first": [int(x) for x in sel[:8]]}
name = "fingerprints_2p32.json" if which == "S0" else f"fingerprints_2p32_{which}.json"
if start:
    name = f"fingerprints_2p32_{which}_at{start}.json"
json.dump(out, open(os.path.join(os.path.dirname(os.path.abspath(__file__)), name), "w"), indent=1)
print(json.dumps(out))
