#!/usr/bin/env python3
"""CPU burn of protocol ranks: run `n` pow_node ranks at a
difficulty where mining takes a while, sample the ranks' CPU use with psutil
for `secs` seconds, print cores used per rank.  Optionally the same for the
reference binary (oracle/_ref/blockchain_ref, fixed d = 9, so its run is short)."""
import os
import signal
import subprocess
import sys
import tempfile
import time

import psutil

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_blockchain_amd.build import build_node  # noqa: E402
from mpi_blockchain_amd.node import MPIEXEC, mpi_env  # noqa: E402


def sample(cmd, secs, cwd):
    p = subprocess.Popen(["timeout", "-k", "5", "60"] + cmd, cwd=cwd, env=mpi_env(),
                         stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, start_new_session=True)
    time.sleep(1.5)  # start-up (HIP init) excluded
    root = psutil.Process(p.pid)
    ranks = [c for c in root.children(recursive=True) if c.name().startswith(("pow_node", "blockchain_ref"))]
    t0 = {r.pid: {t.id: t.user_time + t.system_time for t in r.threads()} for r in ranks}
    time.sleep(secs)
    used = {}
    for r in ranks:
        try:
            # cores used by each thread of the rank, busiest first
            th = {t.id: t.user_time + t.system_time for t in r.threads()}

            def comm(tid):
                try:
                    return open(f"/proc/{r.pid}/task/{tid}/comm").read().strip()
                except OSError:
                    return "?"
            used[r.pid] = sorted(((round((v - t0[r.pid].get(k, 0.0)) / secs, 2), comm(k), k == r.pid)
                                  for k, v in th.items()), reverse=True)[:3]
        except psutil.NoSuchProcess:
            pass
    os.killpg(p.pid, signal.SIGKILL)  # the whole job: launcher, proxies and ranks
    p.wait()
    return used


n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
d = int(sys.argv[2]) if len(sys.argv) > 2 else 34
with tempfile.TemporaryDirectory(ignore_cleanup_errors=True) as td:
    node = os.path.abspath(sys.argv[3]) if len(sys.argv) > 3 else build_node()
    used = sample([MPIEXEC, "-np", str(n), node, "--difficulty", str(d), "--blocks", "100"], 3.0, td)
    print({"ranks": len(used), "difficulty": d, "node": node,
           "cores_per_thread_top3 (cores, name, is_main)": list(used.values())})
