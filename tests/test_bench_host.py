"""Host logic of bench.py that needs no GPU: the live PMC traffic passes
(pmc_traffic_live) parse rocprofv3's counter CSV, drop pow_warmup's empty
dispatch, take the median per sweep dispatch and convert KiB to bytes."""
import csv
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

K1 = "void pow_search<0, false>(PowConsts const*, PowLaunch, unsigned int*, PowResult*)"


def fake_run(values_kib, rc=0, grid=True):
    """A stand-in for subprocess.run that writes what `rocprofv3 --pmc C -d DIR`
    would: one row per (dispatch, counter) in DIR/<host>/<pid>_counter_collection.csv.
    The first dispatch is pow_warmup's one-workgroup launch."""

    def run(cmd, cwd=None, **kw):
        counter = cmd[cmd.index("--pmc") + 1]
        out = os.path.join(cmd[cmd.index("-d") + 1], "host")
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, "1_counter_collection.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"] + (["Grid_Size"] if grid else []))
            for i, v in enumerate(values_kib[counter]):
                w.writerow([i + 1, K1, counter, v] + ([256 if i == 0 else 524032] if grid else []))
            w.writerow([99, "void pow_hash_kernel(unsigned int const*, unsigned int, unsigned int*)", counter, 1e6]
                       + ([64] if grid else []))
        return subprocess.CompletedProcess(cmd, rc, "", "")

    return run


def test_live_traffic_median_without_warmup(monkeypatch):
    monkeypatch.setattr(shutil, "which", lambda name: "/usr/bin/rocprofv3")
    monkeypatch.setattr(bench.os, "access", lambda p, m: True)
    vals = {"FETCH_SIZE": [5.0625, 734.125, 746.8125, 734.0],      # first: pow_warmup's empty launch
            "WRITE_SIZE": [0.125, 71545.90625, 71559.75, 71548.0625]}
    monkeypatch.setattr(bench.subprocess, "run", fake_run(vals))
    r = bench.pmc_traffic_live()
    assert r["FETCH_SIZE"]["kib_per_dispatch"] == [734.0, 734.125, 746.8125]
    assert r["FETCH_SIZE"]["median_bytes"] == int(734.125 * 1024)
    assert r["WRITE_SIZE"]["median_bytes"] == int(71548.0625 * 1024)
    assert r["total_bytes"] == r["FETCH_SIZE"]["median_bytes"] + r["WRITE_SIZE"]["median_bytes"]


def test_live_traffic_robust_to_an_outlier_dispatch(monkeypatch):
    """One sweep dispatch in a few reads tens of MB more (another process on
    the box): the median of the sweeps still holds, with or without the grid
    column, and the warm-up launch is still dropped."""
    monkeypatch.setattr(shutil, "which", lambda name: "/usr/bin/rocprofv3")
    monkeypatch.setattr(bench.os, "access", lambda p, m: True)
    vals = {"FETCH_SIZE": [5.0625, 734.125, 80000.0, 746.8125],
            "WRITE_SIZE": [0.125, 71545.90625, 71559.75, 71548.0625]}
    for grid in (True, False):
        monkeypatch.setattr(bench.subprocess, "run", fake_run(vals, grid=grid))
        r = bench.pmc_traffic_live()
        assert r["FETCH_SIZE"]["kib_per_dispatch"] == [734.125, 746.8125, 80000.0], (grid, r)
        assert r["FETCH_SIZE"]["median_bytes"] == int(746.8125 * 1024)


def test_live_traffic_reports_a_failed_pass(monkeypatch):
    monkeypatch.setattr(shutil, "which", lambda name: "/usr/bin/rocprofv3")
    monkeypatch.setattr(bench.os, "access", lambda p, m: True)
    vals = {"FETCH_SIZE": [734.0], "WRITE_SIZE": [71548.0]}  # too few sweep dispatches
    monkeypatch.setattr(bench.subprocess, "run", fake_run(vals, rc=0))
    r = bench.pmc_traffic_live()
    assert "error" in r and "total_bytes" not in r
    monkeypatch.setattr(bench.subprocess, "run", fake_run({"FETCH_SIZE": [1.0] * 3, "WRITE_SIZE": [1.0] * 3}, rc=137))
    assert "error" in bench.pmc_traffic_live()


def test_live_traffic_without_profiler(monkeypatch):
    monkeypatch.setattr(shutil, "which", lambda name: None)
    assert "error" in bench.pmc_traffic_live()
