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
    # the timed step's own output: its sorted list's sha256 equals the golden fingerprint
    assert d["parity"]["fingerprint_ok"] is True, d["parity"]
    # traffic measured in the run (two rocprofv3 PMC passes): at least the
    # solution list (4 B per solution), at most a few times it
    live = r["counters_live"]
    assert "total_bytes" in live, live
    assert r["traffic"] == live["total_bytes"] and "measured in this run" in r["traffic_source"]
    assert r["algorithmic_bytes"] <= r["traffic"] < 4 * r["algorithmic_bytes"], r
    # the VALU counter pass: ~4,837 VALU instructions per hash, a clock near 2.4 GHz
    assert 4700 < r["valu_instr_per_hash"] < 5000, live
    assert 1.5 < r["measured_clock_ghz"] < 2.5 and 2.0 <= r["cycles_per_valu_instr"] < 6, live
    assert 0 < r["issued_frac_at_measured_clock"] <= r["frac_at_measured_clock"] < 1.0, r
    # no figure labelled "busy" above 100 % (counter_defs' VALUBusy prices SIMD-16 issue)
    assert 0 < r["valu_busy_pct_simd32"] <= 100, r
    assert not [k for k, v in r.items() if "busy" in k and isinstance(v, (int, float)) and v > 100], r


def test_valu_microbench_ceilings():
    """pow_valu_rate: the full-rate chain issues faster than the half-rate one
    (about 2x), each at a measured clock; K1's SHA round stream lies between
    them."""
    import ctypes

    sys.path.insert(0, ROOT)
    import bench
    from mpi_blockchain_amd._lib import POW_VALU_FULL, POW_VALU_HALF, POW_VALU_MIX, ValuResult, load

    L = load()
    out = {}
    for k in (POW_VALU_FULL, POW_VALU_HALF, POW_VALU_MIX):
        r = ValuResult()
        assert L.pow_valu_rate(0, k, ctypes.byref(r)) == 0
        assert 1.0e9 < r.clock_hz < 2.6e9 and r.lane_ops_per_s > 1e12, (k, r.clock_hz, r.lane_ops_per_s)
        out[k] = r
    assert 1.5 < out[POW_VALU_FULL].lane_ops_per_s / out[POW_VALU_HALF].lane_ops_per_s < 2.5
    assert 1.9 < out[POW_VALU_FULL].cycles_per_instr < 2.6 and 3.6 < out[POW_VALU_HALF].cycles_per_instr < 4.6
    # K1's round stream (8 half : 6 full rate) lies between the two (~3.66 in the probes)
    assert out[POW_VALU_FULL].cycles_per_instr < out[POW_VALU_MIX].cycles_per_instr < \
        out[POW_VALU_HALF].cycles_per_instr
    assert L.pow_valu_rate(0, 7, ctypes.byref(ValuResult())) < 0
    # the same measurement on a context's stream (bench.py's form: no extra hardware queue)
    from mpi_blockchain_amd.miner import GpuMiner

    with GpuMiner(0) as m:
        r = ValuResult()
        assert m.L.pow_valu_rate_ctx(m.ctx, POW_VALU_FULL, ctypes.byref(r)) == 0
        assert 0.8 < r.lane_ops_per_s / out[POW_VALU_FULL].lane_ops_per_s < 1.25, r.lane_ops_per_s
        assert 1.9 < r.cycles_per_instr < 2.6
        assert m.L.pow_valu_rate_ctx(None, POW_VALU_FULL, ctypes.byref(r)) < 0


def run_rehearsal(n: int, transport: str = "gloo") -> dict:
    """bench.py as the driver launches it for N > 1 (torch.distributed.run,
    one rank per GPU), rehearsed with n ranks sharing this box's GPU
    (BENCH_REHEARSAL=1; RCCL refuses two ranks on one device).  transport:
    "gloo" (pow_group_init_custom over gloo) or "rccl_stub" (pow_group_init's
    RCCL leg with the test library's shared-memory stand-in for RCCL)."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, BENCH_REHEARSAL="1", BENCH_REHEARSAL_TRANSPORT=transport)
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
                        "--master-addr", "127.0.0.1", "--master-port", str(port),
                        os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "1", "--warmup", "1"],
                       capture_output=True, text=True, timeout=900, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["scaling"] == "weak" and d["value"] > 1e9
    if transport == "gloo":
        assert "gloo all_reduce" in d["config"]["parallelism"] and "pow_group_init_custom" in d["config"]["parallelism"]
    else:
        assert "stand-in RCCL" in d["config"]["parallelism"] and "pow_group_init;" in d["config"]["parallelism"]
    # config 4's cooperative search ran through pow_group's C++ rounds on every
    # rank, and every winner verified (digest, difficulty, range, agreement)
    gs = d["group_search"]
    assert gs["n_gpus"] == n and gs["templates"] == 21 and gs["hashes_all_ranks_mean"] > 0, gs
    assert gs["verified"]["ok"] is True and gs["verified"]["winners_checked"] == 21, gs["verified"]
    assert all(c is not None for c in gs["counters"]), gs
    # the topology block: every rank, the group's own rank count (the stand-in's
    # ncclCommCount), each communicator on its rank's device; one GPU shared
    topo = d["topology"]
    assert [r["rank"] for r in topo["ranks"]] == list(range(n)), topo
    assert all(r["group_comm_count"] == n for r in topo["ranks"]), topo
    assert topo["group_comm_count_ok"] and topo["group_comm_device_ok"] and topo["ok"], topo
    assert topo["rehearsal"] is True and topo["distinct_gpus"] is False, topo  # n ranks, one GPU
    assert topo["group_transport"] == transport
    if transport == "rccl_stub":
        assert topo["rccl_library"].endswith("tests/stub_rccl/libstub_rccl.so"), topo
    assert "cpu_baseline" not in d and "ladder" not in d  # rank-0-at-N=1-only extras
    # per-rank attribution of the step: kernel + all-reduce <= the rank's own step (noise aside)
    tm = d["timing"]
    assert len(tm["per_rank_kernel_ms"]) == n and len(tm["allreduce_ms_per_step"]) == n, tm
    for k, a, st in zip(tm["per_rank_kernel_ms"], tm["allreduce_ms_per_step"], tm["per_rank_step_ms"]):
        assert k > 0 and a > 0 and k + a <= 1.05 * st + 1.0, tm
        assert max(st, k + a) <= 1.05 * d["ms_per_step"] + 1.0, tm  # nobody's step exceeds the job's
    assert tm["imbalance"] >= 1.0 and d["imbalance"] == tm["imbalance"], tm
    assert len(tm["per_rank_clock_ghz"]) == n and all(1.0 < c < 2.6 for c in tm["per_rank_clock_ghz"]), tm
    # the stop board: open and bound on every rank, and peers stopped by it (not at the round's end)
    bd = gs["board"]
    assert [r["rank"] for r in bd["per_rank"]] == list(range(n)), bd
    assert all(r["board_open"] and r["board_bound_every_search"] for r in bd["per_rank"]), bd
    assert bd["all_ranks_board"] is True and bd["stop_latency_samples"] >= 15, bd
    assert bd["peers_stopped_by_board"] is True, bd
    # config 5 at the job's size: mpiexec -np n pow_node (here all on the one GPU)
    pr = d["protocol"]
    assert pr["ranks"] == n
    for key in ("d9", "d25", "d5_forced_fork"):
        assert pr[key]["rc"] == 0 and pr[key]["chains_consistent"] and pr[key]["chains_complete"] >= 1, pr
        assert pr[key]["hard_errors"] == 0, pr
        # every pow_node rank said where it mined: here all on the one GPU (a rehearsal: reported, not failed)
        pl = pr[key]["placement"]
        assert [x["rank"] for x in pl["devices"]] == list(range(n)) and pl["all_ranks_reported"], pl
        assert all(x["device"] == 0 and x["local_rank_from"] == "MPI_LOCALRANKID" for x in pl["devices"]), pl
        assert pl["distinct_gpus"] is False and pl["rehearsal"] is True and pl["ok"] is True, pl
        assert pl["no_local_rank_warnings"] == [], pl
    assert pr["ok"] is True and pr["distinct_gpus"] is False, pr
    assert pr["d5_forced_fork"]["blocks_mined"] >= n and pr["d5_forced_fork"]["fork_events"] >= 1, pr
    return d


def test_bench_multi_rank_rehearsal():
    """2 ranks: rank 0 prints ONE JSON line with n_gpus = 2, the whole-job
    value, and both ranks' windows checked against their fingerprints."""
    d = run_rehearsal(2)
    chk = d["parity"]["checked_ranks"]
    assert d["parity"]["unchecked_ranks"] == [] and d["parity"]["count_ok"] is True, d["parity"]
    assert all(chk[str(r)]["ok"] and chk[str(r)]["fingerprint_ok"] for r in range(2)), chk


FAR = [os.path.join(ROOT, "tests", "golden", f"fingerprints_2p32_S0_at{r << 32}.json") for r in range(1, 8)]


@pytest.mark.skipif(not all(os.path.exists(f) for f in FAR), reason="windows 1..7 fingerprints not all generated")
def test_bench_eight_rank_rehearsal():
    """The driver's 8-GPU launch shape (8 ranks; here sharing one GPU) over
    pow_group_init's RCCL leg (the stand-in RCCL): every rank sweeps its own
    2^32 window, the job total is the sum, and EVERY rank's window
    [r*2^32, (r+1)*2^32) matches the CPU restatement's fingerprints (count,
    lowest counter, sha256 of the timed step's sorted device list)."""
    d = run_rehearsal(8, "rccl_stub")
    chk = d["parity"]["checked_ranks"]
    assert sorted(chk, key=int) == [str(r) for r in range(8)] and d["parity"]["unchecked_ranks"] == [], d["parity"]
    assert all(c["ok"] is True and c["fingerprint_ok"] is True for c in chk.values()), chk
    assert d["parity"]["count_ok"] is True and d["parity"]["fingerprint_ok"] is True
    assert d["parity"]["solutions_all_ranks"] > 8 * 8_000_000


def test_bench_rank_dies_at_group_init():
    """The first N > 1 contact, broken on purpose: rank 1 of 2 dies after its
    GPU set-up, as the group forms (BENCH_TEST_FAIL).  Rank 0, waiting for it
    there, fails or is stopped by torch.distributed.run; both ranks leave their
    `bench_rank_failure` line naming the phase, no result line is printed, and
    the job ends non-zero in seconds, not at the driver's 600 s limit."""
    import socket
    import time

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, BENCH_REHEARSAL="1", BENCH_REHEARSAL_TRANSPORT="rccl_stub", BENCH_TEST_FAIL="1:group_init")
    t = time.monotonic()
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port),
                        os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "1"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    wall = time.monotonic() - t
    assert p.returncode != 0
    fails = {}
    for ln in p.stderr.splitlines():
        if ln.startswith('{"bench_rank_failure"'):
            f = json.loads(ln)["bench_rank_failure"]
            fails[f["rank"]] = f
    assert sorted(fails) == [0, 1], p.stderr[-3000:]
    assert fails[1]["phase"] == "group_init" and fails[1]["exit_code"] == 6, fails[1]
    assert [x[0] for x in fails[1]["phases_done"]] == ["import", "process_group", "device_init"], fails[1]
    # rank 0 waits in the group's id broadcast (or has not got there yet): gloo sees its peer's
    # socket close (exit 6, the collective's error) or torch.distributed.run stops it (SIGTERM, 143)
    assert fails[0]["phase"] in ("process_group", "device_init", "group_init") and \
        fails[0]["exit_code"] in (6, 143), fails[0]
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith('{"metric"')]
    assert wall < 150, wall
