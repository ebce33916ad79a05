"""Run the protocol node (``bin/pow_node``, C++ + MPI) and read its output.

``run_network`` launches an MPI job the way the reference is run
(``mpiexec -np N ./blockchain``, README.md:8-13). It can optionally mix in
ranks of any other binary that speaks the same wire format, e.g. the reference
itself built by ``oracle/Makefile``. ``parse_chain_dump`` reads the
``<rank>.out`` files that log_chain writes (node.cpp:40-58).
"""
from __future__ import annotations

import os
import re
import subprocess
from dataclasses import dataclass, field

from .build import MPI_HOME, NODE_BIN, build_node

MPIEXEC = os.path.join(MPI_HOME, "bin", "mpiexec")


@dataclass
class ChainEntry:
    index: int
    owner: int
    prev: str
    hash: str


@dataclass
class NetworkRun:
    returncode: int
    stdout: str
    chains: dict = field(default_factory=dict)  # rank -> [ChainEntry] (tip first)


def mpi_env() -> dict:
    env = dict(os.environ)
    # MPICH's lib dir also holds an old libstdc++: keep the system one first.
    env["LD_LIBRARY_PATH"] = ":".join(
        p for p in ("/lib/x86_64-linux-gnu", os.path.join(MPI_HOME, "lib"), env.get("LD_LIBRARY_PATH", "")) if p)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def parse_chain_dump(text: str) -> list[ChainEntry]:
    """Blocks of ``Block number / Owner / Previous block hash / Block hash``."""
    out = []
    for m in re.finditer(r"Block number: (\d+)\nOwner: (\d+)\nPrevious block hash: ([^\n]*)\n"
                         r"Block hash: ([^\n]*)\n", text):
        out.append(ChainEntry(int(m.group(1)), int(m.group(2)), m.group(3), m.group(4)))
    return out


def run_network(n_gpu: int, workdir: str, difficulty: int = 9, blocks: int = 10, timeout: float = 240,
                ref_binary: str | None = None, n_ref: int = 0, extra_args=()) -> NetworkRun:
    """mpiexec with n_ref reference ranks (if given) followed by n_gpu GPU ranks."""
    node = build_node()
    if node is None:
        raise RuntimeError("MPI (mpi.h / libmpi.so) not found: cannot build the protocol node")
    args = [node, "--difficulty", str(difficulty), "--blocks", str(blocks), *map(str, extra_args)]
    cmd = [MPIEXEC]
    if n_ref:
        cmd += ["-np", str(n_ref), ref_binary, ":"]
    cmd += ["-np", str(n_gpu), *args]
    p = subprocess.run(["timeout", "-k", "10", str(int(timeout))] + cmd, cwd=workdir, env=mpi_env(),
                       capture_output=True, text=True)
    run = NetworkRun(p.returncode, p.stdout + p.stderr)
    for r in range(n_ref + n_gpu):
        f = os.path.join(workdir, f"{r}.out")
        if os.path.exists(f):
            run.chains[r] = parse_chain_dump(open(f).read())
    return run
