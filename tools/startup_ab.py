"""Config-1 vs config-5 start-up A/B (run on the GPU box): wall time of a
10-block chain at d = 9 with 4 ranks, alternating
  * the reference (mpiexec -np 4 oracle/_ref/blockchain_ref),
  * pow_node with GPU set-up before MPI_Init (--serial-init 1),
  * pow_node with GPU set-up on a thread beside MPI_Init (default),
so drift hits every variant alike.  Prints one JSON line per variant.

    python tools/startup_ab.py [reps]
"""
import json
import os
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpi_blockchain_amd.node import MPIEXEC, mpi_env, run_network  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 7
ref = os.path.join(ROOT, "oracle", "_ref", "blockchain_ref")
walls = {"reference": [], "gpu_serial_init": [], "gpu_overlapped_init": []}
for r in range(reps):
    with tempfile.TemporaryDirectory(ignore_cleanup_errors=True) as td:
        t = time.perf_counter()
        p = subprocess.run(["timeout", "-k", "5", "120", MPIEXEC, "-np", "4", ref], cwd=td, env=mpi_env(),
                           capture_output=True, text=True)
        walls["reference"].append(time.perf_counter() - t)
    for name, extra in (("gpu_serial_init", ("--serial-init", 1)), ("gpu_overlapped_init", ())):
        with tempfile.TemporaryDirectory(ignore_cleanup_errors=True) as td:
            t = time.perf_counter()
            run = run_network(4, td, difficulty=9, blocks=10, timeout=120, extra_args=extra)
            walls[name].append(time.perf_counter() - t)
            assert run.returncode == 0 and run.chains, (name, run.returncode, run.stdout[-2000:])
    print(f"rep {r} done", file=sys.stderr, flush=True)
for name, w in walls.items():
    print(json.dumps({"variant": name, "reps": reps, "wall_s_median": round(statistics.median(w), 3),
                      "wall_s_min": round(min(w), 3), "walls": [round(x, 3) for x in w]}))
