#!/usr/bin/env python3
"""Randomised parity sweep: GPU (through the C ABI) vs the CPU restatement, and
the winner digests vs the reference's own block_to_hash where oracle/_ref is
built.

Each case draws a template (random 32/64-bit header fields, so the reference's
truncation to the low byte is exercised (trap T1); a prev hash that is random
binary, a 64-char hex string + NUL + zeros, a hex string with a non-zero tail
(trap T5), empty, or all 0xFF), a window start (uniform in the counter space,
just below a multiple of 2^32, just below a base-62 carry of nonce char k, or
at the end of the space, 62^9), a window length (2^12..2^19) and a difficulty
(0..14 bits), then checks
  * pow_sweep's solution list == the oracle's (exact, ascending);
  * pow_mine's lowest counter == the list's first (or none);
  * pow_mine_any's counter is in the list;
  * the winner's block_hash == the oracle's (and the reference's) digest, and
    pow_hash_block (K2', one block) gives the same hex.
Stops at the first mismatch (no retries) and prints it.  One JSON summary line.

    python tests/parity_fuzz.py --cases 300 --seed 7      (test infrastructure: it runs the oracle)
    POW_LAT_WPS=4 python tests/parity_fuzz.py --test-hooks --cases 2000 --seed 8   (K1' asm variants)
"""
import argparse
import hashlib
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SPACE = 62 ** 9


def draw(rng: random.Random, k: int):
    idx, own, dif, cat = (rng.randrange(1 << 32), rng.randrange(1 << 32), rng.randrange(1 << 32),
                          rng.randrange(1 << 64))
    kind = k % 5
    if kind == 0:
        prev = bytes(rng.randrange(256) for _ in range(256))
    elif kind == 1:
        prev = hashlib.sha256(rng.randbytes(8)).hexdigest().encode()
    elif kind == 2:  # hex + NUL + a non-zero tail (T5)
        prev = hashlib.sha256(rng.randbytes(8)).hexdigest().encode() + b"\0" + bytes(
            rng.randrange(1, 256) for _ in range(191))
    elif kind == 3:
        prev = b""
    else:
        prev = b"\xff" * 256
    count = rng.randrange(1 << 12, 1 << 19)
    where = rng.randrange(4)
    if where == 0:
        start = rng.randrange(SPACE - count)
    elif where == 1:  # straddle a multiple of 2^32
        m = rng.randrange(1, (SPACE >> 32) - 1) << 32
        start = m - rng.randrange(1, count)
    elif where == 2:  # straddle a carry of nonce char k (62^j counters)
        j = rng.randrange(1, 9)
        m = rng.randrange(1, SPACE // 62 ** j) * 62 ** j
        start = max(0, min(SPACE - count, m - rng.randrange(1, count)))
    else:  # the end of the counter space
        start = SPACE - count
    d = rng.randrange(0, 15)
    return (idx, own, dif, cat, prev), start, count, d


def run(cases: int, seed: int, miner=None, progress=None) -> dict:
    """The cases; returns the summary, or {"mismatch": ...} at the first one."""
    from mpi_blockchain_amd.block import make_block
    from mpi_blockchain_amd.miner import GpuMiner, block_hex
    from oracle.oracle import Oracle, RefLib, make_oblock, ref_available

    O = Oracle()
    ref = RefLib("O2") if ref_available("O2") else None
    threads = min(16, len(os.sched_getaffinity(0)))
    rng = random.Random(seed)
    stats = {"cases": 0, "solutions": 0, "winners_ref_checked": 0, "empty_windows": 0}
    t0 = time.time()
    own = miner is None
    m = GpuMiner(0) if own else miner
    try:
        if own:
            m.warmup()
        for k in range(cases):
            fields, start, count, d = draw(rng, k)
            b = make_block(*fields)
            ob = make_oblock(*fields)
            got = m.sweep(b, start, count, d, cap=count)
            want, n = O.sweep(ob, start, count, d, cap=count, threads=threads)
            case = {"k": k, "start": start, "count": count, "d": d, "prev_kind": k % 5}
            if got.tolist() != want.tolist():
                return {"mismatch": "sweep", **case, "gpu": int(got.size), "oracle": n}
            lo = m.mine(b, start, count, d)
            an = m.mine(b, start, count, d, any_solution=True)
            if want.size == 0:
                stats["empty_windows"] += 1
                if lo is not None or an is not None:
                    return {"mismatch": "mine on an empty window", **case}
            else:
                if lo is None or lo.counter != start + int(want[0]):
                    return {"mismatch": "pow_mine lowest", **case}
                if an is None or (an.counter - start) not in set(want.tolist()):
                    return {"mismatch": "pow_mine_any", **case}
                # the winner's digest: oracle, the reference itself, and K2'
                nonce = O.nonce_from_counter(lo.counter)
                wb = make_oblock(*fields, nonce=nonce)
                _, ohex = O.block_to_hash(wb)
                hx = block_hex(lo.block)
                if hx != ohex or m.block_to_hash(lo.block) != ohex:
                    return {"mismatch": "winner digest", **case, "gpu": hx, "oracle": ohex}
                if ref is not None:
                    if ref.block_to_hash(wb) != ohex:
                        return {"mismatch": "reference digest", **case}
                    stats["winners_ref_checked"] += 1
            stats["cases"] += 1
            stats["solutions"] += int(want.size)
            if progress and (k + 1) % 25 == 0:
                progress(f"{k + 1}/{cases} cases ok ({stats['solutions']} solutions, {time.time() - t0:.0f} s)")
    finally:
        if own:
            m.close()
    stats.update(ok=True, seed=seed, wall_s=round(time.time() - t0, 1), reference=ref is not None)
    return stats


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=300)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--test-hooks", action="store_true",
                    help="run on libpow_gpu_test.so, which reads the test switches (POW_LAT_WPS, POW_FORCE_FULL, "
                         "POW_LAT_MAX) from the environment")
    args = ap.parse_args()
    miner = None
    if args.test_hooks:
        from mpi_blockchain_amd.miner import GpuMiner

        miner = GpuMiner(0, test_hooks=True)
        miner.warmup()
    res = run(args.cases, args.seed, miner=miner, progress=lambda s: print(s, flush=True))
    if miner is not None:
        miner.close()
    print(json.dumps(res), flush=True)
    return 0 if res.get("ok") else 1


if __name__ == "__main__":
    sys.exit(main())
