"""PCIe-inclusive sweep rate: pow_sweep (solution list copied to the host and
returned sorted) vs pow_sweep_device (list stays in HBM; bench.py's form) over
the bench workload (S0, [0, 2^32), d = 9), alternating, in one process.

    python tools/pcie_probe.py --reps 5
"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import WINDOW, s0_block  # noqa: E402
from mpi_blockchain_amd.miner import DeviceBuffer, GpuMiner  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--difficulty", type=int, default=9)
    a = ap.parse_args()
    m = GpuMiner(0)
    tmpl = s0_block()
    cap = 12_000_000
    buf = DeviceBuffer(m, 4 * cap)
    m.sweep_count(tmpl, 0, WINDOW, a.difficulty, dev_out=buf, cap=cap)  # warm-up
    host, dev = [], []
    n_host = n_dev = None
    for i in range(a.reps):
        t0 = time.perf_counter()
        sol = m.sweep(tmpl, 0, WINDOW, a.difficulty, cap=cap)
        host.append(time.perf_counter() - t0)
        n_host = len(sol)
        t0 = time.perf_counter()
        n_dev, _ = m.sweep_count(tmpl, 0, WINDOW, a.difficulty, dev_out=buf, cap=cap)
        dev.append(time.perf_counter() - t0)
        print(f"rep {i + 1}: host-copy {host[-1] * 1e3:.1f} ms ({n_host} solutions, "
              f"{4 * n_host / 1e6:.1f} MB), device {dev[-1] * 1e3:.1f} ms", flush=True)
    assert n_host == n_dev, (n_host, n_dev)
    mh, md = statistics.median(host), statistics.median(dev)
    print(f"median per 2^32 window: host-copy {mh * 1e3:.1f} ms = {WINDOW / mh / 1e9:.3f} G trials/s; "
          f"device {md * 1e3:.1f} ms = {WINDOW / md / 1e9:.3f} G trials/s; "
          f"the copy + host ordering cost {(mh - md) * 1e3:.1f} ms ({(mh / md - 1) * 100:.2f}%)")
    buf.free()
    m.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
