#!/usr/bin/env python3
"""Per-launch fixed cost of the sweep kernel K1 (work-queue tail + launch):
kernel time of a counter sweep of S0 at d = 9 over 2^28 .. 2^32 counters
(median of 5 HIP-event timings each); fit T(n) = n / rate + tail."""
import os
import statistics
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_blockchain_amd.block import make_block  # noqa: E402
from mpi_blockchain_amd.miner import GpuMiner  # noqa: E402

b = make_block(1, 0, 9, 1700000000, b"")
ns, ts = [], []
with GpuMiner(0) as m:
    m.sweep_count(b, 0, 1 << 30, 9)
    for lg in (28, 29, 30, 31, 32):
        t = []
        for _ in range(5):
            m.sweep_count(b, 0, 1 << lg, 9)
            t.append(m.stats()["kernel_ms"])
        ns.append(float(1 << lg))
        ts.append(statistics.median(t))
A = np.vstack([ns, np.ones(len(ns))]).T
(slope, tail), *_ = np.linalg.lstsq(A, np.array(ts), rcond=None)
print({"kernel_ms": dict(zip([28, 29, 30, 31, 32], [round(x, 3) for x in ts])),
       "fit_rate_G_per_s": round(1e-6 / slope, 4), "fit_tail_ms": round(tail, 3)})
