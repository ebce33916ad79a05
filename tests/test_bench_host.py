"""Host logic of bench.py that needs no GPU: the live PMC passes (pmc_live)
parse rocprofv3's counter and kernel-trace CSVs, drop pow_warmup's empty
dispatch, take the median per sweep dispatch, convert KiB to bytes, and derive
VALU instructions per hash, the clock and cycles per instruction; the
roofline block and the CPU-baseline headline."""
import csv
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

K1 = "void pow_search<0, false>(PowConsts const*, PowLaunch, unsigned int*, PowResult*)"


DUR_NS = [1_000, 496_500_000, 496_300_000, 497_000_000]  # first: pow_warmup's launch
VALU = {"SQ_INSTS_VALU": [10.0, 324614173324.0, 324614173640.0, 324614172846.0],
        "SQ_ACTIVE_INST_VALU": [10.0, 324614189694.0, 324614190008.0, 324614189216.0],
        "GRBM_GUI_ACTIVE": [100.0, 9472254275.0, 9473312216.0, 9474333110.0]}


def fake_run(values_kib, rc=0, grid=True):
    """A stand-in for subprocess.run that writes what `rocprofv3 --pmc C.. -d DIR
    [--kernel-trace]` would: one row per (dispatch, counter) in
    DIR/<host>/<pid>_counter_collection.csv (and the kernel trace).  The first
    dispatch is pow_warmup's one-workgroup launch."""

    def run(cmd, cwd=None, **kw):
        i = cmd.index("--pmc") + 1
        counters = []
        while not cmd[i].startswith("-"):
            counters.append(cmd[i])
            i += 1
        out = os.path.join(cmd[cmd.index("-d") + 1], "host")
        os.makedirs(out, exist_ok=True)
        vals = dict(values_kib, **VALU)
        with open(os.path.join(out, "1_counter_collection.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"] + (["Grid_Size"] if grid else []))
            for counter in counters:
                for i, v in enumerate(vals[counter]):
                    w.writerow([i + 1, K1, counter, v] + ([256 if i == 0 else 524032] if grid else []))
                w.writerow([99, "void pow_hash_kernel(unsigned int const*, unsigned int, unsigned int*)", counter,
                            1e6] + ([64] if grid else []))
        if "--kernel-trace" in cmd:
            with open(os.path.join(out, "1_kernel_trace.csv"), "w", newline="") as f:
                w = csv.writer(f)
                w.writerow(["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"])
                for i, dns in enumerate(DUR_NS):
                    w.writerow([i + 1, K1, 1000, 1000 + dns])
        return subprocess.CompletedProcess(cmd, rc, "", "")

    return run


def test_live_traffic_median_without_warmup(monkeypatch):
    monkeypatch.setattr(shutil, "which", lambda name: "/usr/bin/rocprofv3")
    monkeypatch.setattr(bench.os, "access", lambda p, m: True)
    vals = {"FETCH_SIZE": [5.0625, 734.125, 746.8125, 734.0],      # first: pow_warmup's empty launch
            "WRITE_SIZE": [0.125, 71545.90625, 71559.75, 71548.0625]}
    monkeypatch.setattr(bench.subprocess, "run", fake_run(vals))
    r = bench.pmc_live(256)
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
        r = bench.pmc_live(256)
        assert r["FETCH_SIZE"]["kib_per_dispatch"] == [734.125, 746.8125, 80000.0], (grid, r)
        assert r["FETCH_SIZE"]["median_bytes"] == int(746.8125 * 1024)


def test_live_traffic_reports_a_failed_pass(monkeypatch):
    monkeypatch.setattr(shutil, "which", lambda name: "/usr/bin/rocprofv3")
    monkeypatch.setattr(bench.os, "access", lambda p, m: True)
    vals = {"FETCH_SIZE": [734.0], "WRITE_SIZE": [71548.0]}  # too few sweep dispatches
    monkeypatch.setattr(bench.subprocess, "run", fake_run(vals, rc=0))
    r = bench.pmc_live(256)
    assert "error" in r and "total_bytes" not in r
    monkeypatch.setattr(bench.subprocess, "run", fake_run({"FETCH_SIZE": [1.0] * 3, "WRITE_SIZE": [1.0] * 3}, rc=137))
    assert "error" in bench.pmc_live(256)


def test_live_traffic_without_profiler(monkeypatch):
    monkeypatch.setattr(shutil, "which", lambda name: None)
    assert "error" in bench.pmc_live(256)


def test_live_valu_counters(monkeypatch):
    """The third pass: VALU wave-instructions x 64 / 2^32 per hash (r02: 4,837),
    the clock from GRBM_GUI_ACTIVE (summed over 8 XCDs) over the same
    dispatch's duration, cycles per VALU instruction per SIMD."""
    monkeypatch.setattr(shutil, "which", lambda name: "/usr/bin/rocprofv3")
    monkeypatch.setattr(bench.os, "access", lambda p, m: True)
    vals = {"FETCH_SIZE": [5.0, 734.0, 735.0, 736.0], "WRITE_SIZE": [0.1, 71545.0, 71546.0, 71547.0]}
    monkeypatch.setattr(bench.subprocess, "run", fake_run(vals))
    v = bench.pmc_live(256)["valu"]
    assert v["dispatches"] == 3 and v["kernel_ns"] == 496_500_000  # the median duration
    assert abs(v["valu_instr_per_hash"] - 4837.1) < 0.1
    clk = 9472254275.0 / 8 / 0.4965
    assert abs(v["clock_ghz"] - clk / 1e9) < 1e-4
    assert abs(v["cycles_per_valu_instr"] - 1024 * clk * 0.4965 / 324614173324.0) < 1e-3
    r = bench.roofline_block(43.28, 496.2, {"nominal_tops": 78.64}, {"valu": v}, 1, "x", 1, 256)
    assert r["valu_instr_per_hash"] == v["valu_instr_per_hash"]
    assert abs(r["frac_at_measured_clock"] - 43.28 / (1024 * 32 * clk / 1e12)) < 1e-4
    assert 0 < r["issued_frac_at_measured_clock"] < r["frac_at_measured_clock"]
    # with the microbenchmark cycles: K1's mix at the isolated rates over the measured cycles
    peak = {"nominal_tops": 78.64, "microbench_full_rate": {"cycles_per_instr": 2.2},
            "microbench_half_rate": {"cycles_per_instr": 4.2}}
    r = bench.roofline_block(43.28, 496.2, peak, {"valu": v}, 1, "x", 1, 256)
    iso = (bench.TRIAL_HALF_RATE * 4.2 + bench.TRIAL_FULL_RATE * 2.2) / (bench.TRIAL_HALF_RATE + bench.TRIAL_FULL_RATE)
    assert abs(r["isolated_rate_cycles_per_instr"] - iso) < 1e-3
    assert abs(r["issue_efficiency_vs_isolated_rates"] - iso / v["cycles_per_valu_instr"]) < 1e-3


def test_mix_adjusted_ceiling_math():
    """The ceiling prices K1's trial mix at the isolated full- and half-rate
    microbenchmark rates: with the r01 probe's 2.2 / 4.1 cycles at 2.38 GHz it
    is ~9.8 G hashes/s."""
    f_tops = 1024 * 64 * 2.38e9 / 2.2 / 1e12
    h_tops = 1024 * 64 * 2.38e9 / 4.1 / 1e12
    hps = 1.0 / (bench.TRIAL_HALF_RATE / (h_tops * 1e12) + bench.TRIAL_FULL_RATE / (f_tops * 1e12))
    assert 9.7e9 < hps < 9.9e9
    assert bench.TRIAL_HALF_RATE + bench.TRIAL_FULL_RATE == 4839


def test_cpu_baseline_headline_is_the_best_run(monkeypatch):
    """cpu_baseline's value is the best reference rate among the runs (at the
    cgroup quota on the GPU box) and `cores` the CPUs the job can use."""
    import json as _json

    monkeypatch.setattr(bench, "host_cpu_info", lambda: {"affinity": 256, "cgroup_cpu_quota": 16.0,
                                                        "sockets": "2", "cores_per_socket": "64"})
    rates = {("O2", 256): 3.4e6, ("O0", 256): 5.3e5, ("O2", 16): 4.99e6}

    def run(cmd, **kw):
        flav = os.path.basename(cmd[-2])[-2:] if "mpiexec" in cmd[4] else os.path.basename(cmd[0])[-2:]
        np_ = int(cmd[cmd.index("-np") + 1])
        return subprocess.CompletedProcess(cmd, 0, _json.dumps({"ranks": np_, "trials_per_s": rates[(flav, np_)]}), "")

    monkeypatch.setattr(bench.subprocess, "run", run)
    monkeypatch.setattr(bench.os.path, "exists", lambda p: True)
    import mpi_blockchain_amd.build as B
    monkeypatch.setattr(B, "mpi_available", lambda: True)
    r = bench.cpu_baseline()
    assert r["value"] == 4.99e6 and r["cores"] == 16 and r["headline_run"] == "O2_at_quota"
    assert r["value"] >= r["at_cpu_quota"]["value"]
    assert r["logical_cpus"] == 256 and r["physical_cores"] == 128 and r["usable_cpus"] == 16.0
    assert r["as_shipped_O0"] == 5.3e5


def test_launch_plan_branches():
    """--gpus N: no launcher and N > 1 -> launch torch.distributed.run itself;
    a launcher whose WORLD_SIZE differs from N -> refuse; otherwise run."""
    assert bench.launch_plan(1, {}) == "run"
    assert bench.launch_plan(8, {}) == "self"
    assert bench.launch_plan(8, {"WORLD_SIZE": "8"}) == "run"
    assert bench.launch_plan(1, {"WORLD_SIZE": "1"}) == "run"
    assert bench.launch_plan(8, {"WORLD_SIZE": "1"}) == "mismatch"
    assert bench.launch_plan(1, {"WORLD_SIZE": "4"}) == "mismatch"


def test_self_launch_runs_torchrun_as_a_child(monkeypatch, capsys):
    """The self-launch starts torch.distributed.run (one rank per GPU, 127.0.0.1
    rendezvous) as a child process, relays only its JSON line to stdout and
    returns the child's exit code."""
    import io

    seen = {}

    class FakePopen:
        def __init__(self, cmd, stdout=None, text=None, cwd=None):
            seen["cmd"] = cmd
            self.stdout = io.StringIO('[rank0] warming up\n{"metric": "m", "n_gpus": 8}\n[rank3] done\n')

        def wait(self):
            return 7

    monkeypatch.setattr(bench.subprocess, "Popen", FakePopen)
    rc = bench.self_launch(8, ["--gpus", "8", "--steps", "3"])
    cmd = seen["cmd"]
    assert rc == 7
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and cmd[cmd.index("--nproc-per-node") + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1" and "--nnodes=1" in cmd
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"] and cmd[-5].endswith("bench.py")
    out = capsys.readouterr()
    assert out.out == '{"metric": "m", "n_gpus": 8}\n' and "[rank0] warming up" in out.err


def test_main_refuses_a_mismatched_launch(monkeypatch):
    """WORLD_SIZE != --gpus: exit 2 before torch is imported or a GPU is touched."""
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8"])
    import pytest

    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 2


def test_main_self_launches_without_a_launcher(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "1"])
    calls = []
    monkeypatch.setattr(bench, "self_launch", lambda n, argv: calls.append((n, argv)) or 0)
    import pytest

    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0 and calls == [(4, ["--gpus", "4", "--steps", "1"])]


def test_native_group_required_at_n_gt_1():
    """At N > 1 a failed pow_group_init is fatal (no fallback number); at N = 1
    and in the one-GPU rehearsal it is not."""
    assert bench.native_group_error(None, "pow_group_init failed (x)", 8, False) == "pow_group_init failed (x)"
    assert bench.native_group_error(None, None, 2, False) == "pow_group_init failed"
    assert bench.native_group_error(object(), None, 8, False) is None
    assert bench.native_group_error(None, "e", 1, False) is None
    assert bench.native_group_error(None, "e", 8, True) is None


def _topo_rank(r, pci, uuid, count, dev=0, host="h"):
    return {"rank": r, "local_rank": r, "hip_device": dev, "pci": pci, "uuid": uuid, "pid": 100 + r, "host": host,
            "group_comm_count": count, "group_comm_device": dev}


def test_topology_check():
    """The N > 1 record's self-check (bench.topology_check): N distinct GPUs
    by PCI address and UUID, the group's transport counting N ranks, each
    communicator on its rank's device.  A rehearsal (ranks sharing one GPU)
    reports non-distinct GPUs without failing; a real run fails on it."""
    good = [_topo_rank(r, f"0000:{r:02x}:00.0", f"u{r}", 8, dev=r) for r in range(8)]
    t = bench.topology_check(good, 8, "/x/librccl.so", "rccl", False)
    assert t["ok"] and t["distinct_gpus"] and t["group_comm_count_ok"] and t["group_comm_device_ok"]
    shared = [_topo_rank(r, "0000:05:00.0", "u0", 8) for r in range(8)]
    assert not bench.topology_check(shared, 8, None, "rccl", False)["ok"]
    t = bench.topology_check(shared, 8, None, "gloo", True)
    assert t["ok"] and not t["distinct_gpus"]
    short = [dict(x, group_comm_count=4) for x in good]  # RCCL saw 4 ranks in an 8-rank job
    assert not bench.topology_check(short, 8, None, "rccl", False)["ok"]
    wrongdev = [dict(x, group_comm_device=0) for x in good]  # every communicator on GPU 0
    assert not bench.topology_check(wrongdev, 8, None, "rccl", False)["ok"]
    # same PCI address on two hosts is two GPUs
    two_hosts = [_topo_rank(r, "0000:05:00.0", "u0", 2, host=f"h{r}") for r in range(2)]
    assert bench.topology_check(two_hosts, 2, None, "rccl", False)["distinct_gpus"]
    # partitions of one GPU (CPX): one bus and device, distinct functions, possibly one UUID
    cpx = [_topo_rank(r, f"0000:05:00.{r}", "u0", 8, dev=r) for r in range(8)]
    assert bench.topology_check(cpx, 8, None, "rccl", False)["distinct_gpus"]
    missing = [{k: v for k, v in x.items() if k != "group_comm_count"} for x in good]
    assert not bench.topology_check(missing, 8, None, "rccl", False)["ok"]


def _node_line(rank, size, dev, pci, host="h", frm="MPI_LOCALRANKID"):
    return ('pow_node device {"rank": %d, "size": %d, "device": %d, "pci": "%s", "host": "%s", "pid": 1, '
            '"local_rank": %d, "local_rank_from": "%s", "visible_gpus": 8}' % (rank, size, dev, pci, host, rank, frm))


def test_node_placement():
    """Config 5's placement check (bench.node_placement) from pow_node's
    start-up lines: one rank per distinct GPU passes; all ranks on one GPU
    fail a real run and pass a rehearsal; a missing line or a no-local-rank
    warning fails both."""
    good = "\n".join(["[MPI] Lanzando proceso 0"] + [_node_line(r, 8, r, f"0000:{0x05 + r:02x}:00.0")
                                                      for r in range(8)])
    p = bench.node_placement(good, 8, False)
    assert p["ok"] and p["distinct_gpus"] and p["all_ranks_reported"] and [d["device"] for d in p["devices"]] == \
        list(range(8)), p
    shared = "\n".join(_node_line(r, 8, 0, "0000:05:00.0") for r in range(8))
    p = bench.node_placement(shared, 8, False)
    assert not p["ok"] and not p["distinct_gpus"] and "distinct" in p["failed"], p
    assert bench.node_placement(shared, 8, True)["ok"]
    missing = "\n".join(_node_line(r, 8, r, f"0000:{r:02x}:00.0") for r in range(7))
    p = bench.node_placement(missing, 8, False)
    assert not p["ok"] and not p["all_ranks_reported"], p
    warned = "\n".join([_node_line(r, 2, 0, "0000:05:00.0", frm="none") for r in range(2)] +
                       ["pow_node: rank 1 of 2: no node-local rank in the environment (MPI_LOCALRANKID, ...)"])
    p = bench.node_placement(warned, 2, True)
    assert not p["ok"] and p["no_local_rank_warnings"] == [1] and "node-local" in p["failed"], p
    # PCI addresses compare case-insensitively; two hosts with the same address are two GPUs
    two = "\n".join([_node_line(0, 2, 0, "0000:05:00.0", host="a"), _node_line(1, 2, 0, "0000:05:00.0", host="b")])
    assert bench.node_placement(two, 2, False)["ok"]


def test_timing_block():
    """Per-rank attribution of the N > 1 step: kernel, all-reduce, own step,
    what is left of the job's step, and the kernel imbalance (max / min)."""
    ranks = [bench.rank_timing(r, [470.0 + r, 470.0 + r], [0.2, 0.3], 0.4715 * 2, 2) for r in range(4)]
    assert ranks[3] == {"rank": 3, "kernel_ms": 473.0, "allreduce_ms": 0.25, "step_ms": 471.5, "clock_ghz": None}
    with_clk = bench.rank_timing(0, [470.0], [0.2], 0.47, 1, 2.38123)
    assert with_clk["clock_ghz"] == 2.3812 and bench.timing_block([with_clk], 470.5)["per_rank_clock_ghz"] == [2.3812]
    t = bench.timing_block(ranks, 474.0)
    assert t["per_rank_kernel_ms"] == [470.0, 471.0, 472.0, 473.0]
    assert t["allreduce_ms_per_step"] == [0.25] * 4 and t["slowest_kernel_rank"] == 3
    assert abs(t["imbalance"] - 473.0 / 470.0) < 1e-4
    assert t["per_rank_other_ms"][0] == round(474.0 - 470.0 - 0.25, 3)
    one = bench.timing_block([bench.rank_timing(0, [469.5], [], 0.47, 1)], 470.0)
    assert one["imbalance"] == 1.0 and one["allreduce_ms_per_step"] == [0.0]


def test_board_summary():
    """The stop board works when every rank had it bound and peers stop within
    tens of us of the finder; a missing board, or peers that run out their
    shards (~470 ms), say so."""
    ok_rank = {"board_open": True, "board_bound_every_search": True}
    b = bench.board_summary([dict(ok_rank, rank=r) for r in range(8)], [35.0, 40.0, 80.0], 8)
    assert b["all_ranks_board"] and b["peers_stopped_by_board"] and b["stop_latency_us_median"] == 40.0
    # signed: peers that stopped before the finder's host returned
    b = bench.board_summary([dict(ok_rank, rank=r) for r in range(2)], [-12.5, -3.0, 4.0], 2)
    assert b["peers_stopped_by_board"] and b["stop_latency_us_min"] == -12.5 and b["stop_latency_us_median"] == -3.0
    b = bench.board_summary([dict(ok_rank, rank=0), dict(ok_rank, rank=1, board_open=False)], [30.0], 2)
    assert not b["all_ranks_board"] and b["peers_stopped_by_board"] is False
    b = bench.board_summary([dict(ok_rank, rank=r) for r in range(2)], [460_000.0, 470_000.0], 2)
    assert b["all_ranks_board"] and b["peers_stopped_by_board"] is False  # bound, but not stopping peers
    assert bench.board_summary([dict(ok_rank, rank=0)], [], 1)["peers_stopped_by_board"] is None
