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


def test_bench_multi_rank_rehearsal():
    """The N > 1 path as the driver launches it (torch.distributed.run, one
    rank per GPU), rehearsed with 2 ranks sharing this box's GPU over gloo
    (BENCH_REHEARSAL=1; RCCL refuses two ranks on one device): rank 0 prints
    ONE JSON line with n_gpus = 2 and the whole-job value."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, BENCH_REHEARSAL="1")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port),
                        os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "1"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["value"] > 1e9
    assert "gloo all_reduce" in d["config"]["parallelism"]
    assert "cpu_baseline" not in d and "ladder" not in d  # rank-0-at-N=1-only extras
