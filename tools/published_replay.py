"""Replay the reference's own published experiments (BASELINE.md §1,
/root/reference/data/exp: wall time to finish a 10-block chain, median of 5
runs, at d = 5/10/15/18 leading-zero bits with 3/10/20 MPI nodes) with
pow_node mining on this box's GPU.  All ranks share the one GPU (20 ranks
would exceed the box's per-GPU process limit, so that column is skipped).
Process start-up (mpiexec, HIP, MPI_Init) is included, as in the reference's
`time mpiexec ...` runs.  Prints one JSON line per (d, ranks).

    python tools/published_replay.py [runs]
"""
import json
import os
import statistics
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpi_blockchain_amd.node import run_network  # noqa: E402

# reference medians (s); hardware unstated.
PUBLISHED = {(5, 3): 0.103, (5, 10): 0.115, (10, 3): 0.226, (10, 10): 0.161,
             (15, 3): 5.722, (15, 10): 1.588, (18, 3): 44.831, (18, 10): 15.753}

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 5
for (d, n), ref_s in PUBLISHED.items():
    walls, chains_ok = [], True
    for _ in range(runs):
        with tempfile.TemporaryDirectory(ignore_cleanup_errors=True) as td:
            t = time.perf_counter()
            run = run_network(n, td, difficulty=d, blocks=10, timeout=120)
            walls.append(time.perf_counter() - t)
            chains_ok &= run.returncode == 0 and bool(run.chains)
    med = statistics.median(walls)
    print(json.dumps({"difficulty_bits": d, "ranks": n, "blocks": 10, "runs": runs,
                      "gpu_wall_s_median": round(med, 3), "gpu_walls": [round(w, 3) for w in walls],
                      "reference_published_wall_s_median": ref_s, "speedup": round(ref_s / med, 1),
                      "ok": chains_ok}), flush=True)
