#!/usr/bin/env python3
"""Time-to-block probe (BASELINE config 3, lowest rung): median wall time of
pow_mine_any over 201 random templates at difficulty d (default 9), as in
bench.py's ladder.  Run under rocprofv3 --kernel-trace --memory-copy-trace
--stats to split the wall time into kernels and copies."""
import os
import random
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_blockchain_amd.block import make_block  # noqa: E402
from mpi_blockchain_amd.miner import GpuMiner  # noqa: E402

d = int(sys.argv[1]) if len(sys.argv) > 1 else 9
rng = random.Random(1)
with GpuMiner(0) as m:
    times = []
    for _ in range(201):
        b = make_block(rng.randrange(1, 1 << 16), 0, 9, 1700000000 + rng.randrange(256),
                       bytes(rng.randrange(256) for _ in range(32)).hex().encode())
        t = time.perf_counter()
        r = m.mine(b, 0, 1 << 42, d, any_solution=True)
        times.append(time.perf_counter() - t)
    print({"d": d, "ttb_ms_median": round(1e3 * statistics.median(times), 4),
           "ttb_ms_min": round(1e3 * min(times), 4)})
