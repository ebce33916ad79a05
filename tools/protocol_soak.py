"""Protocol soak: many short forking networks of pow_node ranks on one GPU.

Each run is an mpiexec of N GPU ranks at a low difficulty with the fork knobs
of tests/test_node_gpu.py (--winner-pause-us, --pause-us), so lost races,
branch conflicts and chain migrations fire in every run.  A run passes when
mpiexec exits 0 within its time limit, no rank rejects a block as invalid
("Error duro"), and every chain dump a rank wrote is consistent (linked,
consecutive, solving) with at least one complete 10-block chain.

The loop stops at the first failed run (no retries): its output is printed.

    python tools/protocol_soak.py --runs 40 --ranks 8 --difficulty 5
    python tools/protocol_soak.py --runs 40 --ranks 8 --difficulty 5 --forced-fork
    python tools/protocol_soak.py --runs 20 --ranks 2 --ref 2 --difficulty 9   # mixed networks
    python tools/protocol_soak.py --runs 20 --ranks 4 --difficulty 9 --mutual     # mutual chain requests

With --ref K the job also holds K ranks of the REFERENCE's own binary
(oracle/_ref/blockchain_ref, whose difficulty is its macro, 9), as in
tests/test_node_gpu.py::test_mixed_with_reference_nodes.
"""
import argparse
import os
import re
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from mpi_blockchain_amd.node import run_network  # noqa: E402
from test_node_gpu import FORK_MSGS, check_chain  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=40)
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--difficulty", type=int, default=5)
    ap.add_argument("--timeout", type=float, default=60)
    ap.add_argument("--ref", type=int, default=0, help="reference (CPU) ranks in the same job")
    ap.add_argument("--forced-fork", action="store_true",
                    help="--hold-first 1 instead of the timing knobs: every rank mines its own block 1 and "
                         "publishes it after a barrier, so every run must show rival blocks")
    ap.add_argument("--mutual", action="store_true",
                    help="--private-lead 3, as tests/test_node_gpu.py::test_mutual_chain_request: every rank "
                         "must lose by several blocks and splice a peer's chain (find = 2)")
    ap.add_argument("--slow-s", type=float, default=3.0,
                    help="with POW_NODE_LOG_DIR set, keep the output of every run slower than this")
    ap.add_argument("--keep-all", action="store_true", help="with POW_NODE_LOG_DIR set, keep every run's output")
    ap.add_argument("--keep-going", action="store_true", help="count failed runs instead of stopping at the first")
    a = ap.parse_args()
    extra = ("--hold-first", "1") if a.forced_fork else ("--winner-pause-us", "400", "--pause-us", "200")
    if a.mutual:
        extra = ("--private-lead", "3")
    ref = dict(ref_binary=os.path.join(ROOT, "oracle", "_ref", "blockchain_ref"), n_ref=a.ref) if a.ref else {}
    if a.ref:
        if a.difficulty != 9:
            ap.error("the reference binary mines at its DEFAULT_DIFFICULTY macro, 9")
        # as the mixed test: GPU set-up before MPI_Init (reference ranks join no
        # start barrier), and blocks 1-3 left to the reference ranks
        extra = ("--serial-init", "1", "--idle-below", "3")
    walls, forks, failed = [], 0, 0
    for i in range(a.runs):
        with tempfile.TemporaryDirectory(ignore_cleanup_errors=True) as wd:
            t0 = time.perf_counter()
            run = run_network(a.ranks, wd, difficulty=a.difficulty, blocks=10, timeout=a.timeout, extra_args=extra,
                              **ref)
            wall = time.perf_counter() - t0
        ok = run.returncode == 0 and "Error duro" not in run.stdout
        complete = 0
        if ok:
            try:
                complete = sum(check_chain(e, 10, a.difficulty) for e in run.chains.values())
            except AssertionError:
                ok = False
        ok = ok and complete > 0
        n_fork = sum(run.stdout.count(m) for m in FORK_MSGS)
        # a slow network (or any, with --keep-all) keeps its whole output, start-up split included
        keep = os.environ.get("POW_NODE_LOG_DIR")
        if keep and (wall > a.slow_s or a.keep_all):
            os.makedirs(keep, exist_ok=True)
            with open(os.path.join(keep, f"soak_run{i + 1}_wall{wall:.2f}s.log"), "w") as f:
                f.write(f"rc {run.returncode} wall {wall:.3f} s\n{run.stdout}")
        startup = re.findall(r"start line at ([0-9.]+) ms", run.stdout)
        if a.forced_fork:
            ok = ok and n_fork >= 1
        if a.mutual:
            ok = ok and all(f"[{r}] Perdí la carrera por varios contra" in run.stdout and
                            f"[{r}]: find = 2 | received_blockchain_checks = 1" in run.stdout for r in range(a.ranks))
        cross = ""
        if a.ref:  # blocks adopted across implementations (reference ranks are 0..ref-1)
            acc = [(int(r), int(s_)) for r, s_ in
                   re.findall(r"\[(\d+)\] Agregado a la lista bloque con index \d+ enviado por (\d+)", run.stdout)]
            n_rg, n_gr = sum(r < a.ref <= s_ for r, s_ in acc), sum(s_ < a.ref <= r for r, s_ in acc)
            cross = f", ref<-gpu {n_rg}, gpu<-ref {n_gr}"
            ok = ok and n_rg > 0 and n_gr > 0  # blocks crossed the implementations both ways
        forks += n_fork
        walls.append(wall)
        print(f"run {i + 1}/{a.runs}: rc {run.returncode} wall {wall:.2f} s, dumps {len(run.chains)}, "
              f"complete {complete}, fork-path lines {n_fork}{cross}"
              f"{', start line ' + max(startup, key=float) + ' ms' if startup else ''} -> {'ok' if ok else 'FAIL'}",
              flush=True)
        if not ok:
            print(run.stdout[-6000:])
            failed += 1
            if not a.keep_going:
                return 1
    walls.sort()
    verdict = "all passed" if not failed else f"{failed} FAILED"
    print(f"{a.runs} networks of {a.ranks} GPU + {a.ref} reference ranks at d = {a.difficulty}: {verdict}; "
          f"wall median {walls[len(walls) // 2]:.2f} s, max {walls[-1]:.2f} s; "
          f"{sum(w > a.slow_s for w in walls)} slower than {a.slow_s:g} s; {forks} fork-path lines in total")
    return 1 if failed else 0


if __name__ == "__main__":
    sys.exit(main())
