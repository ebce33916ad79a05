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

from .build import MPI_HOME, NODE_TEST_KNOBS, build_node

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
    dumps: dict = field(default_factory=dict)   # rank -> raw bytes of <rank>.out


# A launcher's rank variables (torch.distributed.run sets these in bench.py's
# ranks) must not reach MPI jobs started from such a rank: pow_node takes its
# node-local rank from the MPI launcher's own variables.
_FOREIGN_RANK_VARS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
                      "ROLE_RANK", "ROLE_NAME", "ROLE_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


def mpi_env() -> dict:
    env = {k: v for k, v in os.environ.items()
           if k not in _FOREIGN_RANK_VARS and not k.startswith("TORCHELASTIC_")}
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


def chain_status(entries: list[ChainEntry], blocks: int, difficulty: int) -> tuple[bool, bool]:
    """(consistent, complete) for a logged chain, tip first: consecutive
    indices, each block linked to the next one's hash, every hash solving
    `difficulty` leading zero bits; complete = blocks..1 down to genesis."""
    idx = [e.index for e in entries]
    ok = idx == list(range(idx[0], idx[0] - len(idx), -1)) if idx else True
    ok = ok and all(cur.prev == prev.hash for cur, prev in zip(entries, entries[1:]))
    ok = ok and all(len(e.hash) == 64 and re.fullmatch(r"[0-9a-f]{64}", e.hash) is not None
                    and 256 - int(e.hash, 16).bit_length() >= difficulty for e in entries)
    return ok, ok and idx == list(range(blocks, 0, -1)) and entries[-1].prev == ""


def run_network(n_gpu: int, workdir: str, difficulty: int = 9, blocks: int = 10, timeout: float = 240,
                ref_binary: str | None = None, n_ref: int = 0, extra_args=()) -> NetworkRun:
    """mpiexec with n_ref reference ranks (if given) followed by n_gpu GPU ranks.
    Runs bin/pow_node, or bin/pow_node_test when `extra_args` hold one of the
    protocol tests' race-shaping knobs (build.NODE_TEST_KNOBS)."""
    node = build_node(test=any(str(a) in NODE_TEST_KNOBS for a in extra_args))
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
            raw = open(f, "rb").read()
            run.dumps[r] = raw
            run.chains[r] = parse_chain_dump(raw.decode(errors="replace"))
    return run
