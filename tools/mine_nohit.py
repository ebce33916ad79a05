#!/usr/bin/env python3
"""One pow_mine over S0's first 2^32 counters at a difficulty no counter meets
(56 bits): the mine-mode kernel runs the whole window, writes no solution and
makes only its work-queue atomics (one per 64-prefix chunk per wave) and one
trial-count atomic per wave.  Run under `rocprofv3 --pmc WRITE_SIZE` to price
those atomics in WRITE_SIZE."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_blockchain_amd.block import make_block  # noqa: E402
from mpi_blockchain_amd.miner import GpuMiner  # noqa: E402

with GpuMiner(0) as m:
    r = m.mine(make_block(1, 0, 9, 1700000000, b""), 0, 1 << 32, 56)
    print({"found": r is not None, "stats": m.stats()})
