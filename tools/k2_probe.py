#!/usr/bin/env python3
"""K2 (block_to_hash on the GPU, used for block validation): median kernel time
and call time of pow_hash_block over 200 calls."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_blockchain_amd.block import make_block  # noqa: E402
from mpi_blockchain_amd.miner import GpuMiner  # noqa: E402

b = make_block(3, 1, 9, 1700000000, b"00ab" * 16)
with GpuMiner(0) as m:
    k, w = [], []
    for _ in range(200):
        t = time.perf_counter()
        m.block_to_hash(b)
        w.append(time.perf_counter() - t)
        k.append(m.stats()["kernel_ms"])
    print({"k2_kernel_us_median": round(1e3 * statistics.median(k), 2),
           "call_us_median": round(1e6 * statistics.median(w), 2)})
