"""bench.py keeps the driver's contract: one JSON line with the required keys,
whole-job value, the roofline and parity blocks (short run on one GPU)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_json_contract():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
                        "--no-ladder", "--no-cpu-baseline", "--no-peak", "--no-protocol"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1
    assert d["value"] > 1e9 and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert "workload" in d["config"]
    r = d["roofline"]
    assert r["bound"] and r["peak"] > 0 and 0 < r["frac"] < 1.5
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert d["parity"]["count_ok"] is True
