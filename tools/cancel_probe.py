#!/usr/bin/env python3
"""In-flight cancellation latency (pow_cancel): a search with no solution
(d = 60) over 2^40 counters, cancelled from another thread after 30 ms;
prints the time from the cancel to the return of the mine call, median of 20,
for pow_mine_any and pow_mine, with pow_cancel armed and (for comparison)
without it (the host cancel word alone: the call returns at the end of its
current ~0.13 s launch)."""
import os
import statistics
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_blockchain_amd.block import make_block  # noqa: E402
from mpi_blockchain_amd.miner import GpuMiner  # noqa: E402

b = make_block(5, 1, 9, 1700000000, b"")
out = {}
for armed in (True, False):
    with GpuMiner(0) as m:
        if armed:
            m.cancel()
        for any_solution in (True, False):
            lat = []
            for _ in range(20):
                ep, done = m.epoch, {}

                def run():
                    done["r"] = m.mine(b, 0, 1 << 40, 60, epoch=ep, any_solution=any_solution)
                    done["t"] = time.perf_counter()

                th = threading.Thread(target=run)
                th.start()
                time.sleep(0.03)
                t = time.perf_counter()
                if armed:
                    m.cancel()
                else:
                    m._cancel.value = (m._cancel.value + 1) & 0xFFFFFFFF  # host word only
                th.join()
                assert done["r"] is None
                lat.append(done["t"] - t)
            out[f"{'armed' if armed else 'host_word_only'}_{'any' if any_solution else 'lowest'}_ms"] = \
                round(1e3 * statistics.median(lat), 3)
print(out)
