#!/usr/bin/env python3
"""Protocol diagnostics: run an MPI network of pow_node ranks and timestamp
every output line as it arrives (ms since launch).
    python tools/net_trace.py NP D [extra pow_node args...]"""
import os
import subprocess
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_blockchain_amd.build import build_node  # noqa: E402
from mpi_blockchain_amd.node import MPIEXEC, mpi_env  # noqa: E402

np_, d = sys.argv[1], sys.argv[2]
with tempfile.TemporaryDirectory(ignore_cleanup_errors=True) as td:
    t0 = time.perf_counter()
    p = subprocess.Popen(["timeout", "-k", "5", "120", MPIEXEC, "-np", np_, build_node(), "--difficulty", d,
                          "--blocks", "10", *sys.argv[3:]], cwd=td, env=mpi_env(), stdout=subprocess.PIPE,
                         stderr=subprocess.STDOUT, text=True, bufsize=1)
    for line in p.stdout:
        print(f"{1e3 * (time.perf_counter() - t0):9.2f} {line.rstrip()}", flush=True)
    print("rc", p.wait())
