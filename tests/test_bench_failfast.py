"""An N-rank bench job that breaks must fail fast and say where (bench.RankPhases;
VERDICT r05 next-1): every rank writes one `{"bench_rank_failure": ...}` line
on stderr — its phase, the elapsed times, the reason — and exits non-zero,
whether it raised, ran past a phase budget while blocked inside a C call, or
was stopped by the launcher (SIGTERM) because another rank died.  CPU only:
the failures below happen before any GPU is touched."""
import json
import os
import signal
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# A rank that enters a phase and then blocks inside a C call (libc sleep: the
# main thread does not return to the interpreter, as in pow_group_init).
BLOCKED_RANK = r"""
import ctypes, sys
sys.path.insert(0, %r)
import bench
ph = bench.RankPhases(1, 2, 1).start()
ph.enter("import", 60)
ph.enter("group_init", %s)
print("ready", flush=True)
ctypes.CDLL(None).sleep(60)
"""


def failure_lines(stderr: str) -> list[dict]:
    return [json.loads(ln)["bench_rank_failure"] for ln in stderr.splitlines() if ln.startswith('{"bench_rank_failure"')]


def test_phase_budget_fires_while_blocked_in_c():
    t = time.monotonic()
    p = subprocess.run([sys.executable, "-c", BLOCKED_RANK % (ROOT, "1.5")], capture_output=True, text=True,
                       timeout=60)
    assert p.returncode == 7, (p.returncode, p.stderr[-2000:])
    assert time.monotonic() - t < 30
    (f,) = failure_lines(p.stderr)
    assert f["rank"] == 1 and f["world"] == 2 and f["phase"] == "group_init" and "budget" in f["reason"], f
    assert f["phase_elapsed_s"] >= 1.5 and [x[0] for x in f["phases_done"]] == ["import"], f


def test_sigterm_while_blocked_in_c():
    """torch.distributed.run stops the surviving ranks with SIGTERM: the line
    comes out at once even though the main thread is inside a C call."""
    p = subprocess.Popen([sys.executable, "-c", BLOCKED_RANK % (ROOT, "100")], stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    assert p.stdout.readline().strip() == "ready"
    t = time.monotonic()
    p.send_signal(signal.SIGTERM)
    _, err = p.communicate(timeout=30)
    assert p.returncode == 128 + signal.SIGTERM, (p.returncode, err[-2000:])
    assert time.monotonic() - t < 5
    (f,) = failure_lines(err)
    assert f["phase"] == "group_init" and "SIGTERM" in f["reason"] and f["exit_code"] == 143, f


def test_exception_leaves_its_line():
    env = dict(os.environ, BENCH_TEST_FAIL="0:import")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1"], capture_output=True,
                       text=True, timeout=120, env=env, cwd=ROOT)
    assert p.returncode == 6, (p.returncode, p.stderr[-2000:])
    (f,) = failure_lines(p.stderr)
    assert f["phase"] == "import" and "BENCH_TEST_FAIL" in f["reason"] and "traceback" in f, f
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]  # no result line


def test_rank_dies_before_the_group_forms():
    """2 ranks as the driver launches them: rank 1 dies entering
    init_process_group; rank 0 waits in the rendezvous until
    torch.distributed.run stops it.  Both ranks leave their line, the job
    exits non-zero, well inside the driver's 600 s."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, BENCH_REHEARSAL="1", BENCH_TEST_FAIL="1:process_group")
    t = time.monotonic()
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--steps", "1", "--warmup", "1"], capture_output=True, text=True, timeout=300,
                       env=env, cwd=ROOT)
    wall = time.monotonic() - t
    assert p.returncode != 0
    lines = {f["rank"]: f for f in failure_lines(p.stderr)}
    assert sorted(lines) == [0, 1], p.stderr[-3000:]
    assert lines[1]["phase"] == "process_group" and lines[1]["exit_code"] == 6, lines[1]
    # rank 0 is wherever it had got to (still importing torch, or in the rendezvous) when the launcher stopped it
    assert lines[0]["phase"] in ("import", "process_group") and lines[0]["exit_code"] == 143, lines[0]
    assert wall < 150, wall
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith('{"metric"')]


def test_rank_hangs_before_the_group_forms():
    """2 ranks; rank 1 blocks inside a C call as it enters init_process_group
    (a rank stuck in a driver call: it neither dies nor joins).  With the
    phase budgets scaled down (BENCH_PHASE_SCALE) both ranks fail on their
    own deadlines — rank 1 where it hangs, rank 0 waiting for it in the
    rendezvous, or stopped by the launcher once rank 1 is gone — each with its
    line, and the job ends non-zero in seconds."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, BENCH_REHEARSAL="1", BENCH_TEST_HANG="1:process_group", BENCH_PHASE_SCALE="0.04")
    t = time.monotonic()
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--steps", "1", "--warmup", "1"], capture_output=True, text=True, timeout=300,
                       env=env, cwd=ROOT)
    wall = time.monotonic() - t
    assert p.returncode != 0
    lines = {f["rank"]: f for f in failure_lines(p.stderr)}
    assert sorted(lines) == [0, 1], p.stderr[-3000:]
    # whichever rank's budget runs out first exits 7; the launcher then stops the other (143),
    # unless its own budget fired too
    assert lines[1]["phase"] == "process_group", lines[1]
    assert all(f["phase"] in ("import", "process_group") and f["exit_code"] in (7, 143) for f in lines.values()), lines
    assert any(f["exit_code"] == 7 and "budget" in f["reason"] for f in lines.values()), lines
    assert wall < 60, wall
