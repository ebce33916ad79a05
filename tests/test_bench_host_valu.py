"""bench.py's VALU counter block (CPU only): the busy figure is scaled to the
SIMD-32 issue of gfx950 and cannot exceed 100 %; the raw counter ratio is
reported under a name that does not claim a percentage."""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import bench  # noqa: E402
from test_bench_host import fake_run  # noqa: E402


def test_valu_busy_is_simd32_scaled(monkeypatch):
    monkeypatch.setattr(shutil, "which", lambda name: "/usr/bin/rocprofv3")
    monkeypatch.setattr(bench.os, "access", lambda p, m: True)
    vals = {"FETCH_SIZE": [5.0, 734.0, 735.0, 736.0], "WRITE_SIZE": [0.1, 71545.0, 71546.0, 71547.0]}
    monkeypatch.setattr(bench.subprocess, "run", fake_run(vals))
    v = bench.pmc_live(256)["valu"]
    raw = 324614189694.0 / 256 / (9472254275.0 / 8)
    assert abs(v["sq_active_inst_valu_per_cu_cycle"] - raw) < 1e-3 and raw > 1.0  # the r02-r03 "107-113 %"
    assert abs(v["valu_busy_pct_simd32"] - 50 * raw) < 0.1 and v["valu_busy_pct_simd32"] <= 100
    assert "valu_busy_pct" not in v
    r = bench.roofline_block(43.28, 496.2, {"nominal_tops": 78.64}, {"valu": v}, 1, "x", 1, 256)
    assert not [k for k, x in r.items() if "busy" in k and isinstance(x, (int, float)) and x > 100]
