#!/usr/bin/env python3
"""Benchmark of the MI355X proof-of-work hot path (BASELINE.json metric).

Metric: SHA-256 nonce trials/s (1 trial = the reference's loop body
node.cpp:302-308: nonce -> SHA-256 of the 270-byte block -> leading-zero-bit
test), whole job over N GPUs, plus the achieved fraction of the int32 VALU
roofline.

Workload (BASELINE config 2, one step): the deterministic counter sweep of
2^32 nonces on the fixed synthetic block S0 (index=1, owner=0, difficulty=9,
created_at=1700000000, prev = 256 zero bytes) at difficulty 9 bits; every
solving counter is written to a device buffer (~8.39 M per step).  With N GPUs
each rank sweeps its own 2^32-counter shard [rank*2^32, (rank+1)*2^32) (weak
scaling) and an all-reduce(MIN) of the lowest solving counter + an
all-reduce(SUM) of the counts picks the winner, as a sharded search round
does.  The collectives are the library's own (pow_group_allreduce_u64: RCCL
called from C++, mpi_blockchain_amd/csrc/pow_group.cpp), not torch's.

Config 4's cooperative search is measured beside it (outside the timed
region): `group_search` = time-to-block of pow_group_mine_any over all N GPUs
(every GPU mines a static shard of one template; the first hit stops the
others through the stop board; one all-reduce agrees on the winner).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

Without a launcher, `--gpus N` (N > 1) starts the second form itself as a
child process and relays its JSON line; a launcher's WORLD_SIZE that differs
from --gpus, or a failed pow_group_init at N > 1, exits non-zero.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import statistics
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

OPS_PER_HASH = 5000  # algorithmic int32 VALU ops per trial
WINDOW = 1 << 32


class RankPhases:
    """Where this bench rank is, so that no failure of an N-rank job goes
    unexplained.  The reference's ranks block in MPI_Recv with no bound
    (node.cpp:155-161); a bench rank that hangs the same way (a peer died
    before RCCL's communicator formed, a collective a peer never joins) would
    be killed at the driver's limit with nothing written.  Instead every rank:

    * walks through named phases (import -> process_group -> device_init ->
      group_init -> topology -> warmup -> steps -> parity -> group_search ->
      protocol / report), each with a time budget, under one job deadline
      (BENCH_DEADLINE_S, default 570 s: inside the driver's 600 s limit);
    * on an exception, a phase or job deadline, or SIGTERM (torch.distributed.run
      stops the surviving ranks that way once one rank has failed), writes ONE
      stderr line ``{"bench_rank_failure": {...}}`` — rank, phase, elapsed
      times, the phases done, the reason — and exits non-zero.

    The deadline and signal checks run on a watcher thread, so they fire while
    the main thread is blocked inside a C call (pow_group_init, a collective):
    SIGTERM reaches it through signal.set_wakeup_fd, which the C-level handler
    writes from whichever thread the signal lands on."""

    DEADLINE_S = 570.0
    SIGTERM_REASON = "SIGTERM (the launcher stops the job: another rank failed, or the job was cancelled)"

    def __init__(self, rank: int, world: int, local: int):
        self.rank, self.world, self.local = rank, world, local
        self.t0 = time.monotonic()
        self.phase, self.phase_t0, self.budget = "start", self.t0, None
        self.done: list = []
        self.lock = threading.RLock()  # re-entrant: the SIGTERM handler may run inside enter() on the main thread
        self.emitted = False
        self.deadline = self.t0 + float(os.environ.get("BENCH_DEADLINE_S", self.DEADLINE_S))
        # Tests only: BENCH_TEST_FAIL="<rank>:<phase>" makes that rank raise on
        # entering that phase (a rank that dies before the group forms);
        # BENCH_TEST_HANG="<rank>:<phase>" makes it block there inside a C call
        # (a rank stuck in a driver call); BENCH_PHASE_SCALE scales every phase
        # budget (a hang then fails in seconds).
        self.inject = os.environ.get("BENCH_TEST_FAIL", "")
        self.hang = os.environ.get("BENCH_TEST_HANG", "")
        self.scale = float(os.environ.get("BENCH_PHASE_SCALE", "1"))

    def start(self) -> "RankPhases":
        if threading.current_thread() is threading.main_thread():
            r, w = os.pipe()
            os.set_blocking(w, False)
            # Whichever sees SIGTERM first writes the line: the watcher (through the
            # wakeup fd, while the main thread is blocked in C) or this handler (once
            # the main thread is back in the interpreter, e.g. a sleep the signal cut short).
            signal.signal(signal.SIGTERM, lambda *_: self.abort(128 + signal.SIGTERM, self.SIGTERM_REASON))
            signal.set_wakeup_fd(w, warn_on_full_buffer=False)
            self._rfd = r
        else:  # pragma: no cover - bench.main() always runs on the main thread
            self._rfd = None
        threading.Thread(target=self._watch, name="bench-phase-watch", daemon=True).start()
        return self

    def enter(self, name: str, budget_s: float) -> None:
        with self.lock:
            now = time.monotonic()
            self.done.append([self.phase, round(now - self.phase_t0, 3)])
            self.phase, self.phase_t0, self.budget = name, now, budget_s * self.scale
        if self.inject == f"{self.rank}:{name}":
            raise RuntimeError(f"BENCH_TEST_FAIL: injected failure of rank {self.rank} entering {name}")
        if self.hang == f"{self.rank}:{name}":
            import ctypes

            while True:  # blocked in C, as in a driver call that never returns
                ctypes.CDLL(None).sleep(3600)

    def record(self, reason: str, code: int, **extra) -> dict:
        now = time.monotonic()
        return {"bench_rank_failure": dict(
            rank=self.rank, world=self.world, local_rank=self.local, host=os.uname().nodename, pid=os.getpid(),
            phase=self.phase, phase_elapsed_s=round(now - self.phase_t0, 3), phase_budget_s=self.budget,
            elapsed_s=round(now - self.t0, 3), phases_done=self.done[1:], reason=reason, exit_code=code, **extra)}

    def _emit(self, reason: str, code: int, **extra) -> bool:
        with self.lock:
            if self.emitted:
                return False
            self.emitted = True
            line = json.dumps(self.record(reason, code, **extra))
        try:
            sys.stderr.write(line + "\n")
            sys.stderr.flush()
        except Exception:  # pragma: no cover - stderr gone: the exit code still says it
            pass
        return True

    def fail(self, code: int, reason: str, **extra) -> None:
        """A failure the main thread found: the line, then exit `code` at once
        (os._exit: no atexit teardown of torch's process group or RCCL, which
        could wait for the very peer that failed)."""
        self._emit(reason, code, **extra)
        sys.stdout.flush()
        os._exit(code)

    def abort(self, code: int, reason: str, **extra) -> None:
        """From the watcher (the main thread may be stuck in C) or the SIGTERM
        handler: the line, then _exit without running teardown that could
        block on a stuck GPU.  A second caller (the line is out) waits for the
        first one's _exit."""
        if self._emit(reason, code, **extra):
            os._exit(code)
        time.sleep(5)
        os._exit(code)

    def _watch(self) -> None:
        import select

        while True:
            if self._rfd is not None:
                ready, _, _ = select.select([self._rfd], [], [], 0.25)
                if ready:
                    sigs = os.read(self._rfd, 64)
                    if signal.SIGTERM in sigs:
                        self.abort(128 + signal.SIGTERM, self.SIGTERM_REASON)
            else:  # pragma: no cover
                time.sleep(0.25)
            now = time.monotonic()
            with self.lock:
                over = self.budget is not None and now - self.phase_t0 > self.budget
                phase, budget = self.phase, self.budget
            if over:
                self.abort(7, f"phase '{phase}' ran past its {budget:.0f} s budget (hung?)")
            if now > self.deadline:
                self.abort(7, f"job deadline: {self.deadline - self.t0:.0f} s (BENCH_DEADLINE_S) passed")


def s0_block():
    from mpi_blockchain_amd.block import make_block

    return make_block(1, 0, 9, 1700000000, b"")


def host_cpu_info() -> dict:
    """Host CPUs this process may use: affinity mask, cgroup CPU quota
    (cgroup v2 cpu.max), and lscpu's topology."""
    info = {"os_cpu_count": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except Exception:
        info["affinity"] = os.cpu_count() or 1
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        info["cgroup_cpu_quota"] = None if q == "max" else round(int(q) / int(per), 2)
    except Exception:
        info["cgroup_cpu_quota"] = None
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        keys = {"Model name": "model", "Socket(s)": "sockets", "Core(s) per socket": "cores_per_socket",
                "Thread(s) per core": "threads_per_core", "CPU(s)": "cpus"}
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in keys:
                info[keys[k.strip()]] = v.strip()
    except Exception:
        pass
    return info


def cpu_baseline(seconds: float = 1.5) -> dict | None:
    """The reference's mining loop body (oracle/_ref, compiled from
    /root/reference's own block.cpp + picosha2.h) on ALL host CPUs this job
    may use: one MPI rank per CPU of the affinity mask, launched with
    mpiexec as the reference is (Makefile:24), -O2 and -O0 (as shipped).
    Falls back to one forked process per CPU without MPI, and to the C
    restatement (oracle/liboracle.so) without the reference build."""
    host = host_cpu_info()
    ranks = max(1, host["affinity"])
    quota = host.get("cgroup_cpu_quota")
    usable = min(ranks, quota) if quota else ranks  # CPUs' worth of time the job can get
    out, how = {}, None
    try:
        from mpi_blockchain_amd.build import mpi_available
        from mpi_blockchain_amd.node import MPIEXEC, mpi_env
        use_mpi = mpi_available()
    except Exception:
        use_mpi = False
    # With a CPU quota below the affinity mask, also one rank per CPU of the quota
    # (the reference loop on the CPU time the job actually gets, without throttling).
    runs = [("O2", ranks), ("O0", ranks)]
    if quota and int(quota) < ranks:
        runs.append(("O2_at_quota", max(1, int(quota))))
    for key, np_ in runs:
        flav = key[:2]
        mpi_exe = os.path.join(ROOT, "oracle", "_ref", f"ref_cpu_bench_mpi_{flav}")
        exe = os.path.join(ROOT, "oracle", "_ref", f"ref_cpu_bench_{flav}")
        try:
            if use_mpi and os.path.exists(mpi_exe):
                cmd, how = ["timeout", "-k", "10", "180", MPIEXEC, "-np", str(np_), mpi_exe, str(seconds)], "mpi"
                r = subprocess.run(cmd, capture_output=True, text=True, check=True, env=mpi_env(), cwd="/tmp")
            elif os.path.exists(exe):
                cmd, how = [exe, str(np_), str(seconds)], "fork"
                r = subprocess.run(cmd, capture_output=True, text=True, timeout=180, check=True)
            else:
                continue
            out[key] = json.loads(r.stdout.strip().splitlines()[-1])
        except Exception as e:  # pragma: no cover
            out[key] = {"error": str(e)[-300:]}
    good = {k: v for k, v in out.items() if "trials_per_s" in v and k.startswith("O2")}
    if good:
        # Headline: the best rate the reference loop reaches on this job's CPUs
        # (with a cgroup quota below the affinity mask, 256 ranks throttled onto
        # 16 CPUs' worth of time lose to the at-quota run); `cores` = the CPUs
        # the job can actually use, logical and physical counts beside it.
        key = max(good, key=lambda k: good[k]["trials_per_s"])
        best = good[key]
        nranks = best.get("ranks", best.get("procs", ranks))
        launch = (f"mpiexec -np {nranks} (one MPI rank per CPU{' of the cgroup quota' if key == 'O2_at_quota' else ''})"
                  if how == "mpi" else f"{nranks} forked processes")
        try:
            physical = int(host["sockets"]) * int(host["cores_per_socket"])
        except Exception:
            physical = None
        res = {"value": round(best["trials_per_s"], 1), "unit": "trials/s", "cores": int(round(usable)),
               "kind": "reference",
               "sample": (f"reference proof_of_work loop body (node.cpp:292-308; /root/reference block.cpp + "
                          f"picosha2.h built -O2 by oracle/Makefile), {launch} x {seconds} s, rand() nonces, "
                          f"difficulty 9; the best of the runs in `runs`"),
               "per_core": round(best["trials_per_s"] / max(1.0, usable), 1),
               "logical_cpus": host["affinity"], "physical_cores": physical,
               "usable_cpus": usable, "headline_run": key,
               "runs": {k: ({"ranks": v.get("ranks", v.get("procs")), "trials_per_s": round(v["trials_per_s"], 1)}
                            if "trials_per_s" in v else v) for k, v in out.items()}}
        if "O0" in out and "trials_per_s" in out["O0"]:
            res["as_shipped_O0"] = round(out["O0"]["trials_per_s"], 1)
        if "O2_at_quota" in out and "trials_per_s" in out["O2_at_quota"]:
            q = out["O2_at_quota"]
            res["at_cpu_quota"] = {"ranks": q.get("ranks", q.get("procs")), "value": round(q["trials_per_s"], 1)}
        res["host_cpus"] = dict(host, ranks=ranks, usable=usable)
        return res
    # restatement fallback ("port")
    try:
        import ctypes

        from oracle.oracle import Oracle, make_oblock

        procs = int(max(1, min(ranks, usable)))
        O = Oracle()
        b = make_oblock(1, 0, 9, 1700000000, b"")
        n = 1 << 18
        t = time.perf_counter()
        O.L.oracle_sweep(ctypes.byref(b), 0, n * procs, 9, None, 0, procs)
        dt = time.perf_counter() - t
        return {"value": round(n * procs / dt, 1), "unit": "trials/s", "cores": procs, "kind": "port",
                "sample": f"C restatement (oracle/pow_oracle.c) sweep of {n * procs} counters on {procs} threads",
                "host_cpus": host}
    except Exception as e:  # pragma: no cover
        return {"error": str(e)}


PMC_SUMMARY = os.path.join("profiles", "r02", "final", "pmc_summary.json")


def pmc_traffic_committed():
    """HBM bytes per dispatch of this workload from the committed summary of
    tools/profile_round.sh's rocprofv3 passes (same command and build): the
    fallback when the in-run passes (pmc_live) cannot run."""
    try:
        return int(json.load(open(os.path.join(ROOT, PMC_SUMMARY)))["hbm_bytes_per_dispatch"]["total"])
    except Exception:
        return None


SWEEP_TOOL = os.path.join(ROOT, "tools", "ab_sweep")  # built by __graft_entry__.build()


def _pmc_pass(prof: str, counters: list[str], timeout: float, trace: bool) -> tuple[dict, dict, str]:
    """One rocprofv3 --pmc pass over tools/ab_sweep (S0's 2^32 window at d = 9,
    warm-up + 2 sweeps, this build's libpow_gpu.so).  Per sweep dispatch of
    pow_search<0, false>: {counter: value} and (with `trace`, --kernel-trace in
    the same pass) the duration in ns."""
    import csv
    import glob
    import tempfile

    lib = os.path.join(ROOT, "mpi_blockchain_amd", "libpow_gpu.so")
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        cmd = ["timeout", "-s", "KILL", str(int(timeout)), prof, "--pmc", *counters,
               *(["--kernel-trace"] if trace else []), "-f", "csv",
               "--kernel-include-regex", "pow_search", "-d", td, "-o", "run", "--", SWEEP_TOOL, "2", lib]
        p = subprocess.run(cmd, cwd=td, capture_output=True, text=True, timeout=timeout + 30,
                           env=dict(os.environ, TMPDIR="/tmp"))
        per, grid, dur = {}, {}, {}
        for f in glob.glob(os.path.join(td, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "pow_search<0, false>" in r["Kernel_Name"] and r["Counter_Name"] in counters:
                    d = per.setdefault(r["Dispatch_Id"], {})
                    d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                    grid[r["Dispatch_Id"]] = int(r.get("Grid_Size") or 0)
        for f in glob.glob(os.path.join(td, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "pow_search<0, false>" in r["Kernel_Name"]:
                    dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    # pow_warmup's empty launch of the same kernel (one workgroup) is a dispatch
    # too: keep the full-chip sweeps only (by grid size; without a grid column,
    # drop what is far below the median, not the max: one dispatch in a few reads
    # tens of MB more, r02's pmc_summary.json).
    c0 = counters[0]
    if per and all(grid.values()):
        keep = [k for k in per if grid[k] > 64 * 256]
    else:
        med = sorted(v[c0] for v in per.values())[len(per) // 2] if per else 0.0
        keep = [k for k, v in per.items() if v[c0] >= 0.01 * med]
    keep.sort(key=lambda k: per[k][c0])
    err = "" if p.returncode == 0 and len(keep) >= 3 else \
        (f"{' '.join(counters)} pass rc {p.returncode}, {len(keep)} sweep dispatches: " + (p.stderr or "")[-200:])
    return {k: per[k] for k in keep}, {k: dur[k] for k in keep if k in dur}, err


def pmc_live(cu_count: int, timeout: float = 120) -> dict:
    """Counters of the bench kernel measured now, on this box and build, in
    three rocprofv3 passes (their counters do not fit one pass on gfx950):
      * FETCH_SIZE, then WRITE_SIZE: HBM traffic per dispatch.  Both count KiB
        of 64-B memory-side requests (MI355X_MICROARCH.md, HBM/rocprofv3
        section); the kernel has no wide streaming loads, so FETCH_SIZE needs no
        2x correction.  Median per dispatch of the 3 sweeps.
      * SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU, GRBM_GUI_ACTIVE with the kernel
        trace of the same dispatches: VALU wave-instructions per hash, the
        clock the chip held (GRBM_GUI_ACTIVE is summed over the 8 XCDs) and the
        SIMD cycles per VALU instruction.  The dispatch with the median
        duration."""
    import shutil

    prof = shutil.which("rocprofv3")
    if not prof or not os.access(SWEEP_TOOL, os.X_OK):
        return {"error": "rocprofv3 or tools/ab_sweep missing"}
    out = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        per, _, err = _pmc_pass(prof, [counter], timeout, trace=False)
        if err:
            return {"error": err}
        vals = sorted(v[counter] for v in per.values())
        out[counter] = {"kib_per_dispatch": vals, "median_bytes": int(vals[len(vals) // 2] * 1024)}
    out["total_bytes"] = out["FETCH_SIZE"]["median_bytes"] + out["WRITE_SIZE"]["median_bytes"]
    vc = ["SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE"]
    per, dur, err = _pmc_pass(prof, vc, timeout, trace=True)
    if err or not dur:
        out["valu"] = {"error": err or "no kernel-trace rows"}
        return out
    ks = sorted(dur, key=dur.get)
    k = ks[len(ks) // 2]
    c, t_ns = per[k], dur[k]
    clock = c["GRBM_GUI_ACTIVE"] / 8 / (t_ns * 1e-9)
    out["valu"] = {"counters": c, "kernel_ns": t_ns, "dispatches": len(per),
                   "valu_instr_per_hash": round(c["SQ_INSTS_VALU"] * 64 / WINDOW, 1),
                   "clock_ghz": round(clock / 1e9, 4),
                   # counter_defs.yaml's VALUBusy formula, 100 * SQ_ACTIVE_INST_VALU
                   # / CUs / cycles, prices every VALU instruction at 4 cycles
                   # (SIMD-16) and reads > 100 % on gfx950.  Reported raw (a
                   # ratio, not a percentage) and scaled to the SIMD-32 issue of
                   # a full-rate instruction (2 cycles), which cannot exceed 100 %.
                   "sq_active_inst_valu_per_cu_cycle": round(
                       c["SQ_ACTIVE_INST_VALU"] / cu_count / (c["GRBM_GUI_ACTIVE"] / 8), 4),
                   "valu_busy_pct_simd32": round(
                       50 * c["SQ_ACTIVE_INST_VALU"] / cu_count / (c["GRBM_GUI_ACTIVE"] / 8), 1),
                   "cycles_per_valu_instr": round(4 * cu_count * clock * t_ns * 1e-9 / c["SQ_INSTS_VALU"], 3)}
    return out


K2_TOOL = os.path.join(ROOT, "tools", "ab_k2")  # built by __graft_entry__.build()


def validation_latency() -> dict:
    """The validation hash of a received block (valid_new_block,
    block.cpp:13-25 -> block_to_hash; node.cpp:111-115, 199-253): the call
    median of pow_hash_block (K2', through the C ABI, tools/ab_k2: 3 x 200
    calls on 200 blocks) beside the reference's own block_to_hash timed
    in-process (oracle/_ref, as shipped -O0 and -O2; 2,000 calls)."""
    import ctypes

    out = {}
    lib = os.path.join(ROOT, "mpi_blockchain_amd", "libpow_gpu.so")
    try:
        p = subprocess.run(["timeout", "-k", "5", "120", K2_TOOL, "3", lib], capture_output=True, text=True,
                           check=True)
        g = json.loads(p.stdout.strip().splitlines()[-1])
        out["pow_hash_block_call_us_median"] = g["call_us_median"]
        out["pow_hash_block_call_us_p90"] = g["call_us_p90"]
        out["pow_hash_block_kernel_us_median"] = g["kernel_us_median"]
        out["calls"] = g["calls"]
        from mpi_blockchain_amd.miner import GpuMiner

        with GpuMiner(0) as m:  # how K2' is launched: "hip" (hipLaunchKernel; the shipped library's only path)
            out["launch_path"] = m.launch_path()
    except Exception as e:  # pragma: no cover - reported, not fatal
        out["gpu_error"] = str(e)[-300:]
    try:
        from oracle.oracle import RefLib, make_oblock

        b = make_oblock(3, 0, 9, 1700000000, b"ab" * 32)
        for flav in ("O0", "O2"):
            R = RefLib(flav)
            R.L.ref_block_to_hash_median_ns.restype = ctypes.c_double
            R.L.ref_block_to_hash_median_ns.argtypes = [ctypes.c_void_p, ctypes.c_int]
            out[f"reference_block_to_hash_{flav}_us_median"] = round(
                R.L.ref_block_to_hash_median_ns(ctypes.byref(b), 2000) / 1e3, 2)
    except Exception as e:  # pragma: no cover
        out["reference_error"] = str(e)[-300:]
    g_us = out.get("pow_hash_block_call_us_median")
    for flav in ("O0", "O2"):
        r_us = out.get(f"reference_block_to_hash_{flav}_us_median")
        if g_us and r_us:
            out[f"gpu_call_over_reference_{flav}"] = round(g_us / r_us, 2)
    out["note"] = ("one block per call, as validate_block_for_chain checks a received block; GPU: call = "
                   "hipLaunchKernel + kernel (one wave, ~4,500 dependent VALU instructions) + result in mapped host "
                   "memory; reference: picosha2 + hex on one host core.  The GPU call is SLOWER than the reference's "
                   "block_to_hash (gpu_call_over_reference_O0 / _O2 = how many times the reference's as-shipped "
                   "-O0 / -O2 time): f3 keeps one authoritative SHA-256 implementation on both sides of the wire, "
                   "it is not a speed-up")
    return out


def protocol_runs() -> dict:
    """BASELINE config 1 (the reference: mpiexec -np 4 ./blockchain, 10 blocks
    at DEFAULT_DIFFICULTY = 9, picosha2 on CPU) beside config 5 scaled to this
    GPU (4 pow_node ranks, same protocol, GPU mining): wall time to a
    10-block chain, process start-up included."""
    import tempfile

    out = {}
    try:
        from mpi_blockchain_amd.build import mpi_available
        from mpi_blockchain_amd.node import MPIEXEC, mpi_env, run_network

        if not mpi_available():
            return {"skipped": "no MPI"}
        ref = os.path.join(ROOT, "oracle", "_ref", "blockchain_ref")
        if os.path.exists(ref):
            with tempfile.TemporaryDirectory(ignore_cleanup_errors=True) as td:
                t = time.perf_counter()
                p = subprocess.run(["timeout", "-k", "5", "120", MPIEXEC, "-np", "4", ref], cwd=td,
                                   env=mpi_env(), capture_output=True, text=True)
                out["reference_np4_d9_wall_s"] = round(time.perf_counter() - t, 3)
                out["reference_rc"] = p.returncode
        # config 1 at d = 17 (oracle/Makefile: the reference with
        # block.h's DEFAULT_DIFFICULTY line set to 17) for an aggregate CPU rate:
        # 10 blocks x 2^17 expected trials / wall.  Each reference rank busy-polls a
        # second core in MPI_Recv: 4 ranks occupy 8 CPUs.
        ref17 = os.path.join(ROOT, "oracle", "_ref", "blockchain_ref_d17")
        if os.path.exists(ref17):
            with tempfile.TemporaryDirectory(ignore_cleanup_errors=True) as td:
                t = time.perf_counter()
                p = subprocess.run(["timeout", "-k", "5", "120", MPIEXEC, "-np", "4", ref17], cwd=td,
                                   env=mpi_env(), capture_output=True, text=True)
                w = time.perf_counter() - t
                out["reference_np4_d17_wall_s"] = round(w, 3)
                out["reference_np4_d17_rc"] = p.returncode
                out["reference_np4_d17_trials_per_s_est"] = round(10 * 2 ** 17 / w, 1)
        else:
            out["reference_np4_d17"] = "unmeasured: oracle/_ref/blockchain_ref_d17 not built"
        for d in (9, 17, 25):
            with tempfile.TemporaryDirectory(ignore_cleanup_errors=True) as td:
                t = time.perf_counter()
                run = run_network(4, td, difficulty=d, blocks=10, timeout=180)
                out[f"gpu_np4_d{d}_wall_s"] = round(time.perf_counter() - t, 3)
                out[f"gpu_np4_d{d}_rc"] = run.returncode
                out[f"gpu_np4_d{d}_chains"] = len(run.chains)
        # The reference's own published experiment closest to real mining
        # (d = 18, 3 nodes, 10 blocks, median 44.831 s on
        # unstated hardware); tools/published_replay.py replays the whole table.
        with tempfile.TemporaryDirectory(ignore_cleanup_errors=True) as td:
            t = time.perf_counter()
            run = run_network(3, td, difficulty=18, blocks=10, timeout=180)
            out["gpu_np3_d18_wall_s"] = round(time.perf_counter() - t, 3)
            out["gpu_np3_d18_rc"] = run.returncode
            out["reference_published_np3_d18_wall_s"] = 44.831
    except Exception as e:  # pragma: no cover
        out["error"] = str(e)
    return out


def wait_for_exit(pids, timeout: float) -> bool:
    """True once none of `pids` (this node's other bench ranks) is alive
    (a zombie waiting for the launcher to reap it holds no GPU)."""
    t = time.time()
    while time.time() - t < timeout:
        alive = 0
        for pid in pids:
            try:
                with open(f"/proc/{pid}/stat") as f:
                    alive += f.read().rsplit(")", 1)[1].split()[0] != "Z"
            except OSError:
                pass
        if not alive:
            return True
        time.sleep(0.05)
    return False


FORK_EVENTS = ("Perdí la carrera", "Conflicto suave", "Conflicto de branch", "TAG_CHAIN_HASH")


def node_placement(output: str, world: int, rehearsal: bool) -> dict:
    """Where the ranks of one `mpiexec -np N pow_node` job mined: the
    `pow_node device {...}` line each rank writes to stderr at start-up
    (HIP device, PCI address, host, and which launcher variable chose the
    device), and the ranks that warned that no node-local rank was set.
    At N > 1 on real GPUs every rank must sit on its own GPU (distinct host +
    PCI address); in a rehearsal (ranks sharing one GPU by design) that is
    reported, not required."""
    import re

    devs = {}
    for m in re.finditer(r"^pow_node device (\{.*\})\s*$", output, re.M):
        try:
            d = json.loads(m.group(1))
            devs[d["rank"]] = d
        except (ValueError, KeyError):
            continue
    warned = sorted(int(m.group(1)) for m in re.finditer(r"^pow_node: rank (\d+) of \d+: no node-local rank", output,
                                                          re.M))
    ranks = [devs[r] for r in sorted(devs)]
    distinct = len({(d.get("host"), str(d.get("pci", "")).lower()) for d in ranks}) == world and len(ranks) == world
    complete = sorted(devs) == list(range(world))
    ok = complete and not warned and (distinct or rehearsal)
    out = {"devices": [{k: d.get(k) for k in ("rank", "device", "pci", "host", "local_rank", "local_rank_from")}
                       for d in ranks],
           "distinct_gpus": distinct, "all_ranks_reported": complete, "no_local_rank_warnings": warned,
           "rehearsal": rehearsal, "ok": ok}
    if not ok:
        out["failed"] = ("not every rank reported its device" if not complete else
                         "ranks without a node-local rank (all on GPU 0)" if warned else
                         f"{world} ranks on fewer than {world} distinct GPUs")
    return out


def protocol_job(world: int, timeout: float = 90, rehearsal: bool = False) -> dict:
    """BASELINE config 5 at the job's size: `mpiexec -np N pow_node`, one MPI
    rank per GPU of this node (pow_node binds node-local rank r to GPU r), the
    reference's protocol (broadcast, validation, chain migration) with GPU
    mining, 10 blocks.  Run by rank 0 after the timed region while the other
    bench ranks wait idle.  d = 9 (the reference's DEFAULT_DIFFICULTY), d = 25
    (real mining: 10 x 2^25 expected trials) and d = 5 with a forced fork
    (--hold-first: every rank mines its own block 1, published after a
    barrier, so every rank must resolve rival blocks).  Each network's
    `placement` shows the GPU every rank mined on (node_placement); at N > 1
    on real GPUs a network whose ranks do not sit on N distinct GPUs is marked
    failed (`ok` false), as is the whole block."""
    import re
    import tempfile

    from mpi_blockchain_amd.build import mpi_available
    from mpi_blockchain_amd.node import chain_status, run_network

    if not mpi_available():
        return {"skipped": "no MPI"}
    out = {"ranks": world, "blocks": 10}
    for key, d, extra in (("d9", 9, ()), ("d25", 25, ()), ("d5_forced_fork", 5, ("--hold-first", "1"))):
        try:
            with tempfile.TemporaryDirectory(ignore_cleanup_errors=True) as td:
                t = time.perf_counter()
                run = run_network(world, td, difficulty=d, blocks=10, timeout=timeout, extra_args=extra)
                wall = time.perf_counter() - t
            st = [chain_status(c, 10, d) for c in run.chains.values()]
            out[key] = {"wall_s": round(wall, 3), "rc": run.returncode,
                        "chains_consistent": all(ok for ok, _ in st), "chains_complete": sum(c for _, c in st),
                        "blocks_mined": len(re.findall(r"Agregué un producido", run.stdout)),
                        "fork_events": sum(run.stdout.count(m) for m in FORK_EVENTS),
                        "hard_errors": run.stdout.count("Error duro"),
                        "placement": node_placement(run.stdout, world, rehearsal)}
        except Exception as e:  # pragma: no cover - reported, not fatal
            out[key] = {"error": str(e)[-300:]}
    nets = [out[k] for k in ("d9", "d25", "d5_forced_fork")]
    out["distinct_gpus"] = all(n.get("placement", {}).get("distinct_gpus") for n in nets)
    out["ok"] = all("error" not in n and n["rc"] == 0 and n["placement"]["ok"] for n in nets)
    if not out["ok"]:
        out["failed"] = "; ".join(f"{k}: " + (n.get("error") or (f"rc {n['rc']}" if n["rc"] else n["placement"].get(
            "failed", ""))) for k, n in zip(("d9", "d25", "d5_forced_fork"), nets)
                                  if "error" in n or n["rc"] or not n["placement"]["ok"])
    return out


def ladder(miner, n_templates: int = 101, rungs=(9, 13, 17, 21, 25)) -> dict:
    """BASELINE config 3: time-to-block (median over templates, seed 1) and
    sustained hashes/s per difficulty rung.  Time-to-block uses pow_mine_any
    (first solution found, as a miner wants); pow_mine's lowest-counter form
    is the deterministic parity mode."""
    import random

    from mpi_blockchain_amd.block import make_block

    rng = random.Random(1)
    out = {}
    base = s0_block()
    for d in rungs:
        times, hashes = [], []
        for _ in range(n_templates):
            b = make_block(rng.randrange(1, 1 << 16), 0, 9, 1700000000 + rng.randrange(256),
                           bytes(rng.randrange(256) for _ in range(32)).hex().encode())
            t = time.perf_counter()
            r = miner.mine(b, 0, 1 << 42, d, any_solution=True)
            times.append(time.perf_counter() - t)
            hashes.append(r.hashes if r else 0)
        t = time.perf_counter()
        ks = 0.0
        for _ in range(2):
            miner.sweep_count(base, 0, WINDOW, d)
            ks += miner.stats()["kernel_ms"]
        wall = time.perf_counter() - t
        out[str(d)] = {"time_to_block_ms_median": round(1e3 * statistics.median(times), 3),
                       "time_to_block_ms_p90": round(1e3 * sorted(times)[int(0.9 * len(times))], 3),
                       "expected_hashes": 2 ** d,
                       "hashes_median": int(statistics.median(hashes)),
                       "sustained_hashes_per_s": round(2 * WINDOW / wall, 1),
                       "kernel_hashes_per_s": round(2 * WINDOW / (ks * 1e-3), 1)}
    return out


BOARD_STOP_OK_US = 50_000  # a peer that ran out its shard instead (2^32 counters) takes ~470,000 us


def board_summary(per_rank: list[dict], stop_us: list[float], world: int) -> dict:
    """Did the stop board work?  Per rank: the group has the node's board and
    every search ran bound to it; across ranks: the stop latency of each
    search with a finder (the last rank's mine return minus the finder's,
    CLOCK_MONOTONIC on one node).  With a board that is missing or not coherent
    across GPUs the peers only stop at the round's all-reduce, after their
    whole shard: the latency is then hundreds of ms, not tens of us.  It is
    signed: the peers' kernels see the finder's hit on the board as its kernel
    stores it, so they can return before the finder's own host has seen it."""
    out = {"per_rank": per_rank,
           "all_ranks_board": all(r["board_open"] and r["board_bound_every_search"] for r in per_rank),
           "stop_latency_samples": len(stop_us)}
    if world == 1:
        out["stop_latency_us_median"] = None
        out["peers_stopped_by_board"] = None
        out["note"] = "one rank: no peers to stop"
        return out
    if stop_us:
        med = statistics.median(stop_us)
        out["stop_latency_us_median"] = round(med, 1)
        out["stop_latency_us_min"] = round(min(stop_us), 1)
        out["stop_latency_us_max"] = round(max(stop_us), 1)
        out["peers_stopped_by_board"] = out["all_ranks_board"] and med < BOARD_STOP_OK_US
    else:
        out["stop_latency_us_median"] = None
        out["peers_stopped_by_board"] = None
    out["note"] = ("stop latency = when the last peer's pow_mine_any returned (a rank that found nothing) minus "
                   "when the finder's did (CLOCK_MONOTONIC, one node), per search with both; negative = the peers "
                   "stopped before the finder's host saw its own hit; peers_stopped_by_board needs every rank bound "
                   f"to the board and a median under {BOARD_STOP_OK_US} us (a peer that runs out its 2^32-counter "
                   "shard takes ~470 ms)")
    return out


def group_search(group, rank: int, world: int, d: int = 30, n_templates: int = 21, gather=None) -> dict:
    """BASELINE config 4, cooperative form: time-to-block of pow_group_mine_any
    over every GPU of the job (collective; the same templates on every rank).
    Each rank mines its static shard; the first hit stops the node's other
    GPUs inside their launches (stop board) and one all-reduce agrees on the
    winner.  Expected trials per block 2^d; strong scaling in N.

    Every winner is verified (outside the timed calls): its nonce is the
    counter's, its digest recomputed by pow_hash_block is the block_hash it
    carries and solves d (solves_problem, block.cpp:91-96), the counter lies in
    the searched range, and every rank reports the same counter (all-reduce
    min == max).  The verdicts are all-reduced too, so every rank sees the
    same `verified` block."""
    import random

    from mpi_blockchain_amd.block import field, make_block, nonce_from_counter, solves_problem
    from mpi_blockchain_amd.miner import block_hex

    U64MAX = (1 << 64) - 1
    span = 1 << 48
    rng = random.Random(1)
    times, hashes, counters = [], [], []
    stop_us, mine_ms, ar_ms, rounds = [], [], [], []
    bound_every, found = True, 0
    bad = {"no_winner": 0, "nonce": 0, "digest": 0, "solves": 0, "range": 0, "ranks_disagree": 0}
    for _ in range(n_templates):
        b = make_block(rng.randrange(1, 1 << 16), 0, 9, 1700000000 + rng.randrange(256),
                       bytes(rng.randrange(256) for _ in range(32)).hex().encode())
        group.allreduce([0], "sum")  # line the ranks up
        t = time.perf_counter()
        r = group.mine(b, 0, span, d, any_solution=True)
        times.append(time.perf_counter() - t)
        info = group.last_search()  # this rank's part (pow_group_last_search)
        bound_every = bound_every and bool(info["board_bound"])
        found += info["local_found"]
        mine_ms.append(info["mine_ms"])
        ar_ms.append(info["allreduce_ms"])
        rounds.append(info["rounds"])
        # the finder's return (the first, if several found) and the last peer's (a rank that found nothing)
        fin = group.allreduce([info["mine_end_ns"] if info["local_found"] else U64MAX], "min")[0]
        peer_end = group.allreduce([0 if info["local_found"] else info["mine_end_ns"]], "max")[0]
        if fin != U64MAX and peer_end and world > 1:
            stop_us.append((peer_end - fin) / 1e3)  # signed: < 0 = the peers stopped before the finder returned
        hashes.append(group.allreduce([r.hashes if r else 0], "sum")[0])
        c = r.counter if r else U64MAX
        counters.append(r.counter if r else None)
        lo, hi = group.allreduce([c], "min")[0], group.allreduce([c], "max")[0]
        v = [0] * 6
        if r is None:
            v[0] = 1
        else:
            hx = block_hex(r.block)
            v[1] = int(field(r.block, "nonce") != nonce_from_counter(c))
            v[2] = int(group.miner.block_to_hash(r.block) != hx)
            v[3] = int(not solves_problem(hx, d))
            v[4] = int(not 0 <= c < span)
        v[5] = int(lo != hi)
        for k, x in zip(bad, group.allreduce(v, "max")):
            bad[k] += x
    tot_t = sum(times)
    mine_info = {"rank": rank, "board_open": bool(info["board_open"]), "board_bound_every_search": bound_every,
                 "searches_found_here": found, "mine_ms_mean": round(statistics.mean(mine_ms), 3),
                 "allreduce_ms_mean": round(statistics.mean(ar_ms), 3), "rounds_max": max(rounds)}
    per_rank = (gather or (lambda o: [o]))(mine_info)
    verified = {"winners_checked": n_templates, "failures": bad, "ok": not any(bad.values()),
                "how": "nonce == counter's, pow_hash_block(winner) == its block_hash, solves_problem(hash, d), "
                       "0 <= counter < 2^48, all-reduce(min) == all-reduce(max) of the ranks' counters"}
    return {"difficulty_bits": d, "templates": n_templates, "n_gpus": world,
            "time_to_block_ms_median": round(1e3 * statistics.median(times), 3),
            "time_to_block_ms_mean": round(1e3 * tot_t / n_templates, 3),
            "expected_hashes": 2 ** d, "hashes_all_ranks_mean": int(sum(hashes) / n_templates),
            "hashes_per_s_all_ranks": round(sum(hashes) / tot_t, 1),
            "counters": counters, "verified": verified, "board": board_summary(per_rank, stop_us, world),
            "note": "pow_group_mine_any over all GPUs (static shards, stop board, one all-reduce per round); "
                    "hashes include the trials peers ran before the winner's hit reached them"}


def rank_topology(rank: int, local: int, group, miner) -> dict:
    """What this rank ran on: its HIP device, the device's full PCI address
    (domain:bus:device.function, pow_device_pci_bus_id: partitions of one GPU
    differ in the function) and UUID (torch.cuda.get_device_properties), and
    RCCL's own view of the group's communicator (pow_group_info:
    ncclCommCount, ncclCommCuDevice)."""
    import torch

    p = torch.cuda.get_device_properties(local)
    out = {"rank": rank, "local_rank": local, "hip_device": local, "pci": miner.pci_bus_id().lower(),
           "uuid": str(p.uuid), "pid": os.getpid(), "host": os.uname().nodename}
    if group is not None:
        try:
            out.update({f"group_{k}": v for k, v in group.info().items()})
        except Exception as e:  # pragma: no cover - reported; the check below fails on it
            out["group_info_error"] = str(e)[-200:]
    return out


def topology_check(ranks: list[dict], world: int, rccl_library: str | None, transport: str,
                   rehearsal: bool) -> dict:
    """The N > 1 record's self-check: N distinct GPUs (full PCI address per
    host), the group's transport counting N ranks, and each rank's
    communicator on the rank's own device.  UUIDs are reported (partitions of
    one GPU may share one).  In a rehearsal the ranks share one GPU by design:
    distinctness is reported, not required."""
    pcis = {(r["host"], r["pci"]) for r in ranks}
    distinct = len(pcis) == world
    counts = [r.get("group_comm_count") for r in ranks]
    count_ok = all(c == world for c in counts)
    dev_ok = all(r.get("group_comm_device") == r["hip_device"] for r in ranks)
    ok = count_ok and dev_ok and (distinct or rehearsal)
    return {"ranks": ranks, "distinct_gpus": distinct, "group_comm_count_ok": count_ok,
            "group_comm_device_ok": dev_ok, "group_transport": transport, "rccl_library": rccl_library,
            "ok": ok, "rehearsal": rehearsal}


# Issue classes of one trial of K1's j-loop (4,839 VALU instructions, read from
# the gfx950 ISA; tests/test_build.py checks these against the disassembly):
# half rate = 2,046 v_alignbit_b32 + 719 v_add3_u32 + 9 otherwise full-rate ops
# with an SGPR operand; full rate = v_bitop3_b32, v_add_u32, v_lshrrev_b32, ...
TRIAL_HALF_RATE = 2774
TRIAL_FULL_RATE = 2065


def valu_peaks(miner, device: int, cu_count: int) -> dict:
    """Measured ceilings (pow_valu_rate, include/pow_tools.h; every stream 8-byte
    encodings at K1's code phase): the full-rate chain (v_bitop3_b32 +
    v_add_u32_e64, the SIMD-32 ceiling), the half-rate chain (v_alignbit_b32 +
    v_add3_u32), and K1's SHA-256 round stream alone (no schedule words), each
    with the clock the chip held; and the mix-adjusted ceiling: K1's trial mix
    (TRIAL_*_RATE) issued at the two isolated rates, priced at 5,000
    algorithmic ops per hash."""
    import ctypes

    from mpi_blockchain_amd._lib import POW_VALU_FULL, POW_VALU_HALF, POW_VALU_MIX, ValuResult

    out = {}
    for name, kind in (("full_rate", POW_VALU_FULL), ("half_rate", POW_VALU_HALF), ("sha_round", POW_VALU_MIX)):
        r = ValuResult()
        if miner.L.pow_valu_rate_ctx(miner.ctx, kind, ctypes.byref(r)) == 0:  # on the miner's stream: no extra queue
            out[f"microbench_{name}"] = {"tops": round(r.lane_ops_per_s / 1e12, 2),
                                         "clock_ghz": round(r.clock_hz / 1e9, 4),
                                         "cycles_per_instr": round(r.cycles_per_instr, 3)}
    f, h = out.get("microbench_full_rate"), out.get("microbench_half_rate")
    if f and h:
        hps = 1.0 / (TRIAL_HALF_RATE / (h["tops"] * 1e12) + TRIAL_FULL_RATE / (f["tops"] * 1e12))
        out["mix_adjusted_ceiling_tops"] = round(hps * OPS_PER_HASH / 1e12, 2)
        out["mix_adjusted_ceiling_hashes_per_s"] = round(hps, 1)
        out["measured_clock_ghz"] = f["clock_ghz"]
        out["peak_at_measured_clock_tops"] = round(cu_count * 4 * 32 * f["clock_ghz"] * 1e9 / 1e12, 2)
    return out


def roofline_block(achieved, kms, peak, live, traffic, traffic_source, algo_bytes, cu_count) -> dict:
    """The roofline object of the bench line (int32 VALU issue bound)."""
    r = {"bound": "valu_int32", "achieved": round(achieved, 3), "peak": peak["nominal_tops"],
         "unit": "Tops/s", "frac": round(achieved / peak["nominal_tops"], 4),
         "traffic": traffic, "algorithmic_bytes": algo_bytes, "ops_per_hash": OPS_PER_HASH,
         "peak_detail": peak, "traffic_source": traffic_source,
         "note": ("achieved = 2^32 hashes x 5000 int32 ops / mean HIP-event kernel time; peak = 256 CU x 4 SIMD "
                  "x 32 lanes x nominal clock; traffic = FETCH_SIZE+WRITE_SIZE bytes per dispatch of the same "
                  "workload")}
    if "mix_adjusted_ceiling_tops" in peak:
        r["frac_of_mix_adjusted_ceiling"] = round(achieved / peak["mix_adjusted_ceiling_tops"], 4)
        r["frac_of_full_rate_microbench"] = round(achieved / peak["microbench_full_rate"]["tops"], 4)
    if live is not None:
        r["counters_live"] = live
        v = live.get("valu", {})
        if "clock_ghz" in v:
            peak_clk = cu_count * 4 * 32 * v["clock_ghz"] * 1e9 / 1e12
            r["valu_instr_per_hash"] = v["valu_instr_per_hash"]
            r["valu_busy_pct_simd32"] = v["valu_busy_pct_simd32"]
            r["sq_active_inst_valu_per_cu_cycle"] = v["sq_active_inst_valu_per_cu_cycle"]
            r["cycles_per_valu_instr"] = v["cycles_per_valu_instr"]
            r["measured_clock_ghz"] = v["clock_ghz"]
            r["frac_at_measured_clock"] = round(achieved / peak_clk, 4)
            # VALU lane-ops the counters saw issued, over the same kernel's duration in the pass
            r["issued_frac_at_measured_clock"] = round(
                v["counters"]["SQ_INSTS_VALU"] * 64 / (v["kernel_ns"] * 1e-9) / 1e12 / peak_clk, 4)
            # Issue efficiency, clock-free: K1's trial mix priced at the isolated
            # per-instruction cycles of the two microbenchmark streams, over the
            # cycles per VALU instruction the counters measured (1.0 = no mixing cost)
            f, h = peak.get("microbench_full_rate"), peak.get("microbench_half_rate")
            if f and h and v.get("cycles_per_valu_instr"):
                iso = ((TRIAL_HALF_RATE * h["cycles_per_instr"] + TRIAL_FULL_RATE * f["cycles_per_instr"])
                       / (TRIAL_HALF_RATE + TRIAL_FULL_RATE))
                r["isolated_rate_cycles_per_instr"] = round(iso, 3)
                r["issue_efficiency_vs_isolated_rates"] = round(iso / v["cycles_per_valu_instr"], 4)
    return r


def list_fingerprint(buf, n: int) -> str:
    """sha256 of the ascending solution list (little-endian u32), the form of
    tests/golden/fingerprints_2p32*.json: the device list is copied once and
    sorted on the host (after the timed region)."""
    import hashlib

    import numpy as np

    a = np.sort(buf.read_u32(n))
    return hashlib.sha256(a.astype("<u4").tobytes()).hexdigest()


def launch_plan(gpus: int, env) -> str:
    """How this process runs `bench.py --gpus N`:
      * "run"      — it is one rank already (WORLD_SIZE set by the launcher and
                     equal to N), or N = 1;
      * "self"     — N > 1 and no launcher: start torch.distributed.run with N
                     ranks as a CHILD process (before torch or the GPU is
                     touched; no exec) and relay its JSON line;
      * "mismatch" — a launcher started this rank for a job of a different
                     size than --gpus: measuring it would mislabel n_gpus."""
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return "self" if gpus > 1 else "run"
    return "run" if int(ws) == gpus else "mismatch"


def self_launch(gpus: int, argv: list[str]) -> int:
    """`python bench.py --gpus N` without a launcher: run the driver's own
    launch shape (torch.distributed.run, one rank per GPU, rendezvous on
    127.0.0.1) as a child, pass its JSON line through on stdout (everything
    else to stderr), and return its exit code."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, cwd=ROOT)
    for line in p.stdout:
        if line.startswith("{"):
            print(line, end="", flush=True)
        else:
            sys.stderr.write(line)
    return p.wait()


def native_group_error(group, group_err: str | None, world: int, rehearsal: bool) -> str | None:
    """At N > 1 the per-step collectives and config 4's search must run through
    the library's own group (RCCL from C++); a job whose pow_group_init failed
    on any rank stops with this message instead of measuring a fallback."""
    if world > 1 and not rehearsal and group is None:
        return group_err or "pow_group_init failed"
    return None


def rank_timing(rank: int, kernel_ms: list, allreduce_ms: list, own_wall_s: float, steps: int,
                clock_ghz: float | None = None) -> dict:
    """One rank's timed steps: mean HIP-event kernel ms per step, mean wall ms
    in the step's two all-reduces (pow_group_allreduce_u64; waiting for slower
    peers included), the rank's own wall ms per step before the closing
    barrier, and the shader clock its GPU held under load right after them
    (clock_ghz: pow_valu_rate_ctx's K1-mix probe, run by every rank at once)."""
    return {"rank": rank,
            "kernel_ms": round(statistics.mean(kernel_ms), 3) if kernel_ms else None,
            "allreduce_ms": round(statistics.mean(allreduce_ms), 3) if allreduce_ms else 0.0,
            "step_ms": round(1e3 * own_wall_s / max(1, steps), 3),
            "clock_ghz": round(clock_ghz, 4) if clock_ghz else None}


def loaded_clock_ghz(miner) -> float | None:
    """The shader clock this rank's GPU holds under the K1 instruction mix,
    measured on the miner's stream (pow_valu_rate_ctx, POW_VALU_MIX; ~0.1 s).
    Every rank runs it at the same moment, so at N > 1 it is the clock under
    the whole node's load: a GPU whose clock droops shows here."""
    import ctypes

    from mpi_blockchain_amd._lib import POW_VALU_MIX, ValuResult

    r = ValuResult()
    if miner.L.pow_valu_rate_ctx(miner.ctx, POW_VALU_MIX, ctypes.byref(r)) != 0 or r.clock_hz <= 0:
        return None
    return r.clock_hz / 1e9


def timing_block(ranks: list[dict], ms_per_step: float) -> dict:
    """The N > 1 line's attribution of its step time: per rank kernel,
    all-reduce and own-step ms, the kernel imbalance (max / min over ranks:
    one slow GPU shows as > 1), and per rank what is left of the job's step
    (ms_per_step, the slowest rank's wall) after kernel + all-reduce: host time
    and waiting at the closing barrier."""
    ks = [r["kernel_ms"] for r in ranks if r.get("kernel_ms")]
    return {"per_rank_kernel_ms": [r.get("kernel_ms") for r in ranks],
            "allreduce_ms_per_step": [r.get("allreduce_ms") for r in ranks],
            "per_rank_step_ms": [r.get("step_ms") for r in ranks],
            "per_rank_other_ms": [round(ms_per_step - (r.get("kernel_ms") or 0) - (r.get("allreduce_ms") or 0), 3)
                                  for r in ranks],
            "imbalance": round(max(ks) / min(ks), 4) if ks and min(ks) > 0 else None,
            "per_rank_clock_ghz": [r.get("clock_ghz") for r in ranks],
            "slowest_kernel_rank": max(ranks, key=lambda r: r.get("kernel_ms") or 0)["rank"] if ranks else None,
            "note": "kernel = HIP-event time of the step's sweep; allreduce = wall time of its two "
                    "pow_group_allreduce_u64 calls (min, sum), waiting for peers included; other = ms_per_step "
                    "minus both; clock = the shader clock each GPU held under the K1 mix, all ranks at once, "
                    "right after the timed steps"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--difficulty", type=int, default=9)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ladder", action="store_true")
    ap.add_argument("--no-peak", action="store_true")
    ap.add_argument("--no-protocol", action="store_true")
    ap.add_argument("--no-group-search", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the live rocprofv3 traffic passes")
    args = ap.parse_args()

    plan = launch_plan(args.gpus, os.environ)
    if plan == "self":
        sys.exit(self_launch(args.gpus, sys.argv[1:]))
    if plan == "mismatch":
        print(f"bench.py: --gpus {args.gpus} but the launcher started a job of WORLD_SIZE="
              f"{os.environ.get('WORLD_SIZE')}", file=sys.stderr)
        sys.exit(2)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ph = RankPhases(rank, world, local).start()
    try:
        run_rank(args, ph, world, rank, local)
    except SystemExit:
        raise
    except BaseException as e:  # every rank's failure leaves its line: which phase, why
        import traceback

        ph.fail(6, f"exception: {type(e).__name__}: {str(e)[-400:]}",
                traceback=traceback.format_exc(limit=6)[-1500:])


def run_rank(args, ph: RankPhases, world: int, rank: int, local: int) -> None:
    """One bench rank, phase by phase (RankPhases)."""
    ph.enter("import", 240)  # the first `import torch` on a fresh box pages the image in (1-2 min)
    import torch

    dist = None
    rehearsal = os.environ.get("BENCH_REHEARSAL") == "1"
    if world > 1 or "TORCHELASTIC_RUN_ID" in os.environ or os.environ.get("BENCH_FORCE_DIST") == "1":
        import datetime

        import torch.distributed as dist

        # A peer that never joins fails the rendezvous and torch's collectives
        # in 120 s, inside the driver's 600 s limit (torch's default is ~10 min).
        ph.enter("process_group", 150)
        pg_timeout = datetime.timedelta(seconds=120)
        # BENCH_REHEARSAL=1 (tests only): several ranks share the visible
        # GPU(s) and talk over gloo, to exercise the N > 1 path on a one-GPU
        # box (RCCL refuses two ranks on one device).  The numbers it prints
        # are not a scaling measurement.
        if rehearsal:
            dist.init_process_group("gloo", timeout=pg_timeout)
            local = local % max(1, torch.cuda.device_count())
            torch.cuda.set_device(local)
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=pg_timeout)

    ph.enter("device_init", 120)
    from mpi_blockchain_amd.miner import DeviceBuffer, GpuMiner
    from mpi_blockchain_amd.shard import RcclGroup, ShardedMiner, rccl_path

    # A rehearsal (ranks sharing one GPU; tests only) runs the same pow_group
    # rounds with the all-reduce either over gloo (pow_group_init_custom;
    # BENCH_REHEARSAL_TRANSPORT=gloo, the default) or through pow_group_init's
    # RCCL leg with the test library's shared-memory stand-in for RCCL
    # (rccl_stub: tests/stub_rccl): RCCL itself refuses two ranks on one GPU.
    transport = os.environ.get("BENCH_REHEARSAL_TRANSPORT", "gloo") if rehearsal else "rccl"
    if transport == "rccl_stub":
        from mpi_blockchain_amd.build import STUB_LIB

        os.environ["POW_TEST_RCCL_LIB"] = STUB_LIB
    miner = GpuMiner(local, test_hooks=transport == "rccl_stub")
    # The library's own RCCL communicator (the id travels over torch.distributed);
    # at N = 1 a one-rank group, used only by the group_search measurement.
    # pow_group_init gives up after 60 s if a peer never joins (RCCL's init on
    # a helper thread under a deadline).
    ph.enter("group_init", 120)
    group, group_err = None, None
    if transport == "gloo":
        group = ShardedMiner(miner, rank, world)
    else:
        try:
            group = RcclGroup.from_torch(miner) if dist is not None else \
                RcclGroup(miner, 0, 1, RcclGroup.make_unique_id(miner.L))
        except Exception as e:  # fatal at N > 1 (below); at N = 1 only group_search is lost, said in group_error
            group_err = f"pow_group_init failed ({e})"
            group = None
        if dist is not None:
            # Every rank uses the native group or none does (a rank that lacks it
            # would leave its peers waiting in the group's collectives).
            ok = torch.tensor([1 if group is not None else 0], dtype=torch.int64,
                              device="cpu" if rehearsal else f"cuda:{local}")
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if int(ok.item()) == 0 and group is not None:
                group.close()
                group = None
                group_err = "pow_group_init failed on a peer rank"
        err = native_group_error(group, group_err, world, transport == "gloo")
        if err:  # fail loudly: no N > 1 number without the native collectives
            ph.fail(3, "bench.py: no native pow_group at N > 1", group_error=err)
    # Who took part: every rank's GPU (PCI address, UUID) and the group's own
    # count of ranks (RCCL: ncclCommCount), gathered before anything is timed.
    # At N > 1 a record that cannot show N distinct GPUs under one N-rank
    # communicator is not measured: every rank exits non-zero.
    ph.enter("topology", 60)
    topo_ranks = [rank_topology(rank, local, group, miner)]
    if dist is not None:
        topo_ranks = [None] * world
        dist.all_gather_object(topo_ranks, rank_topology(rank, local, group, miner))
    rlib = None
    if transport != "gloo":
        try:
            rlib = rccl_path(miner.L)
        except Exception as e:  # pragma: no cover
            rlib = f"unknown ({e})"
    topology = topology_check(topo_ranks, world, rlib, transport, rehearsal)
    if world > 1 and not topology["ok"]:
        ph.fail(4, "bench.py: topology check failed at N > 1", topology=topology)
    info = miner.device_info()
    tmpl = s0_block()
    d = args.difficulty
    start = rank * WINDOW
    cap = 12_000_000  # > 2^32 / 2^9 * 1.4
    buf = DeviceBuffer(miner, 4 * cap)
    if dist is not None and group is None:
        red = torch.zeros(2, dtype=torch.int64, device="cpu" if rehearsal else f"cuda:{local}")

    kernel_ms, allreduce_ms = [], []

    local_last = [None]  # this rank's (solutions, lowest counter) of the last step

    def step():
        n, mn = miner.sweep_count(tmpl, start, WINDOW, d, dev_out=buf, cap=cap)
        kernel_ms.append(miner.stats()["kernel_ms"])
        local_last[0] = (n, mn)
        if dist is not None and group is not None:  # RCCL through pow_group_allreduce_u64
            a0 = time.perf_counter()
            lo = group.allreduce([mn if mn is not None else (1 << 64) - 1], "min")[0]
            tot = group.allreduce([n], "sum")[0]
            allreduce_ms.append(1e3 * (time.perf_counter() - a0))
            return tot, lo
        if dist is not None:  # rehearsal (several ranks share one GPU over gloo), or no native group
            a0 = time.perf_counter()
            red[0] = mn if mn is not None else (1 << 63) - 1
            dist.all_reduce(red[0:1], op=dist.ReduceOp.MIN)
            red[1] = n
            dist.all_reduce(red[1:2], op=dist.ReduceOp.SUM)
            out = int(red[1].item()), int(red[0].item())
            allreduce_ms.append(1e3 * (time.perf_counter() - a0))
            return out
        return n, mn

    ph.enter("warmup", 60 + 30 * args.warmup)
    first = None
    for _ in range(args.warmup):
        first = step()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    kernel_ms.clear()
    allreduce_ms.clear()
    ph.enter("steps", 60 + 30 * args.steps)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        last = step()
    torch.cuda.synchronize()
    el_own = time.perf_counter() - t0  # this rank's own steps, before it waits for the others
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist is not None:
        tt = torch.tensor([el], dtype=torch.float64, device="cpu" if rehearsal else f"cuda:{local}")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())

    # Per-rank parity (outside the timed region): every rank's window whose
    # fingerprints are committed (rank 0: [0, 2^32); rank 7: [7*2^32, 8*2^32),
    # the farthest window of an 8-GPU run) is checked against them.  With it,
    # each rank's own timing: its mean kernel ms and all-reduce ms per step and
    # its own steps' wall (a sub-linear N > 1 result is attributable from the
    # record: one slow GPU, the collective, or host time between them).
    ph.enter("parity", 120)
    n_loc = local_last[0][0]
    local_last[0] = (*local_last[0], list_fingerprint(buf, n_loc) if d == 9 and n_loc <= cap else None)
    if dist is not None:
        dist.barrier()  # every GPU loaded at once for the clock probe
    my_timing = rank_timing(rank, kernel_ms, allreduce_ms, el_own, args.steps, loaded_clock_ghz(miner))
    per_rank = [(local_last[0], my_timing)]
    if dist is not None:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, (local_last[0], my_timing))
    timing = timing_block([t for _, t in per_rank], 1e3 * el / args.steps)
    per_rank = [p for p, _ in per_rank]
    gsearch = None
    if group is not None and not args.no_group_search:
        ph.enter("group_search", 300)

        def gather(obj):
            if dist is None:
                return [obj]
            out = [None] * world
            dist.all_gather_object(out, obj)
            return out

        try:
            gsearch = group_search(group, rank, world, gather=gather)
        except Exception as e:  # pragma: no cover - reported, not fatal: the headline is measured
            gsearch = {"error": str(e)[-300:]}
        # A winner that does not verify (identical verdict on every rank: all-reduced)
        # makes an N > 1 record unusable: exit non-zero like a missing group.
        if world > 1 and "verified" in gsearch and not gsearch["verified"]["ok"]:
            ph.fail(5, "bench.py: group_search winners failed verification", verified=gsearch["verified"])
    # Config 5 on this job's GPUs: rank 0 launches the MPI job once every
    # other bench rank has exited (their processes release the GPUs, so each
    # GPU carries one pow_node rank and at most bench rank 0 besides).
    proto = None
    do_proto = dist is not None and world > 1 and not args.no_protocol
    pids = None
    if do_proto:
        pids = [None] * world
        dist.all_gather_object(pids, os.getpid())
    # Every rank releases the library's communicator at the same point, before
    # rank 0 goes on alone to config 5: RCCL's teardown of a multi-rank
    # communicator may wait for its peers' (ncclCommFinalize is "globally
    # quiescent"), so ranks 1..N-1 must not be left waiting in it for rank 0.
    had_group = group is not None
    if group is not None and dist is not None:
        ph.enter("group_close", 60)
        group.close()
        group = None
    if rank != 0:
        ph.enter("teardown", 60)
        buf.free()
        if group is not None:
            group.close()
        dist.destroy_process_group()
        return
    if do_proto:
        ph.enter("protocol_wait", 150)
        gone = wait_for_exit(pids[1:], timeout=120)
        ph.enter("protocol", 360)
        proto = protocol_job(world, rehearsal=rehearsal) if gone else \
            {"skipped": "bench ranks 1..N-1 did not exit within 120 s"}
    ph.enter("report", 480)
    collective = ("gloo all_reduce(min,sum) per step via pow_group_allreduce_u64 (pow_group_init_custom; "
                  "rehearsal: ranks share one GPU)" if transport == "gloo" and rehearsal and had_group else
                  "stand-in RCCL (tests/stub_rccl, shared memory) all_reduce(min,sum) per step via "
                  "pow_group_allreduce_u64 (pow_group_init; rehearsal: ranks share one GPU)"
                  if transport == "rccl_stub" and had_group else
                  "rccl all_reduce(min,sum) per step via pow_group_allreduce_u64" if had_group and world > 1
                  else f"{dist.get_backend()} all_reduce(min,sum) per step via torch.distributed" if dist is not None
                  else "none (single process)")

    kms = statistics.mean(kernel_ms) if kernel_ms else float("nan")
    value = world * WINDOW * args.steps / el
    achieved = WINDOW * OPS_PER_HASH / (kms * 1e-3) / 1e12  # Tops/s of the dominant kernel
    clock_ghz = info["clock_khz"] / 1e6
    peak_nominal = info["cu_count"] * 4 * 32 * clock_ghz * 1e9 / 1e12  # SIMD-32: 128 lane-ops/CU/clk
    peak = {"nominal_tops": round(peak_nominal, 2), "nominal_clock_ghz": clock_ghz, "cu_count": info["cu_count"]}
    if not args.no_peak:
        peak.update(valu_peaks(miner, local, info["cu_count"]))
    # Counters of the dominant kernel: live rocprofv3 PMC passes at N = 1 (a
    # child process per pass, after the timed region): HBM traffic, and the VALU
    # instruction / busy / clock counters; the committed summary of the same
    # traffic passes otherwise, labelled as such.
    traffic, traffic_source, live = None, None, None
    if world == 1 and d == 9 and not args.no_pmc:
        try:
            live = pmc_live(info["cu_count"])
        except Exception as e:  # pragma: no cover - reported, not fatal
            live = {"error": str(e)[-300:]}
        if "total_bytes" in live:
            traffic = live["total_bytes"]
            traffic_source = ("measured in this run: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE passes "
                              "(child processes, tools/ab_sweep over S0's 2^32 window at d = 9 with this build), "
                              "median per dispatch of 3")
    if traffic is None:
        traffic = pmc_traffic_committed()
        traffic_source = (f"{PMC_SUMMARY} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this command, "
                          "median per dispatch; not measured in this run)")
    # sanity/parity at full size: rank 0's window is the golden 2^32 window
    parity = {"solutions_rank0": per_rank[0][0], "solutions_all_ranks": last[0], "lowest": last[1]}
    checked = {}
    for r, (n_r, mn_r, fp_r) in enumerate(per_rank):
        fpp = os.path.join(ROOT, "tests", "golden",
                           "fingerprints_2p32.json" if r == 0 else f"fingerprints_2p32_S0_at{r * WINDOW}.json")
        if d == 9 and os.path.exists(fpp):
            want = json.load(open(fpp))["ladder"]["9"]
            checked[str(r)] = {"solutions": n_r, "expected": want["count"],
                               "ok": n_r == want["count"] and mn_r == r * WINDOW + want["first"][0],
                               "fingerprint_ok": fp_r == want["sha256_le_u32"]}
    parity["unchecked_ranks"] = [r for r in range(world) if str(r) not in checked]
    if checked:
        parity["checked_ranks"] = checked
        parity["count_ok"] = all(c["ok"] for c in checked.values())
        parity["fingerprint_ok"] = all(c["fingerprint_ok"] for c in checked.values())
        parity["fingerprint"] = ("sha256 of each checked rank's sorted solution list (the timed step's device "
                                 "output) vs tests/golden/fingerprints_2p32*.json")
    res = {
        "metric": "SHA-256 nonce trials/sec (whole job) + % int32 VALU peak",
        "value": round(value, 1),
        "unit": "trials/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * el / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic",
        "config": {"workload": "counter-nonce sweep of 2^32 nonces per GPU on fixed block S0, "
                               f"difficulty {d} bits (BASELINE config 2; config 4 when N>1)",
                   "template": "S0", "counters_per_gpu_per_step": WINDOW, "difficulty_bits": d,
                   "parallelism": f"static nonce shards x{world}; collective: {collective}"},
        "hashes_per_s_per_gpu": round(value / world, 1),
        "kernel_ms_per_step": round(kms, 3),
        "timing": timing,
        "imbalance": timing["imbalance"],
        "roofline": roofline_block(achieved, kms, peak, live, traffic, traffic_source, 4 * (last[0] or 0),
                                   info["cu_count"]),
        "device": info,
        "parity": parity,
        "topology": topology,
    }
    if world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline()
    if world == 1 and not args.no_ladder:
        res["ladder"] = ladder(miner)
    if gsearch is not None:
        res["group_search"] = gsearch
    if group_err:
        res["group_error"] = group_err
    if world == 1 and not args.no_protocol:
        res["protocol"] = protocol_runs()
        res["protocol"]["validation_hash"] = validation_latency()
    if proto is not None:
        res["protocol"] = proto
    print(json.dumps(res), flush=True)
    ph.enter("teardown", 60)
    buf.free()
    if group is not None:
        group.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
