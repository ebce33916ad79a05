"""Protocol runs (BASELINE config 5, scaled to one GPU): MPI networks of
``pow_node`` ranks mining on the GPU through pow_mine, and mixed networks with
the REFERENCE's own binary (oracle/_ref/blockchain_ref, built from
/root/reference) — the reference's picosha2 validation (valid_new_block,
block.cpp:13-25) accepting GPU-mined blocks is the wire-level parity check.
"""
import os
import re
import time

import pytest

from helpers import check_chain
from mpi_blockchain_amd.build import mpi_available
from mpi_blockchain_amd.node import run_network

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not mpi_available(), reason="no MPI in this image")]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_BIN = os.path.join(ROOT, "oracle", "_ref", "blockchain_ref")


FORK_MSGS = ("Perdí la carrera", "Conflicto suave", "TAG_CHAIN_HASH")
# A rival block 1 received while this rank's chain is at index 1 (node.cpp:235)
# or already past it (node.cpp:242): the fork --hold-first forces.
RIVAL_BLOCK1 = re.compile(r"Conflicto suave: (Conflicto de branch \(1\)|Descarto el bloque \(1 vs \d+\))")


@pytest.mark.parametrize("np_, d", [(4, 9), (6, 5), (8, 5)])  # protocol smoke at d = 5, -np 8
def test_gpu_network(tmp_path, np_, d):
    # Every rank starts mining at the same start line (the MPI_Barrier after
    # GPU set-up in pow_node's main).  At d = 5 the fork is forced rather
    # than left to timing: --hold-first makes every rank mine block 1 and
    # publish it only after a barrier, so every rank receives rival blocks 1.
    extra = ("--hold-first", "1") if d <= 5 else ()
    t0 = time.perf_counter()
    run = run_network(np_, str(tmp_path), difficulty=d, blocks=10, timeout=240, extra_args=extra)
    if os.environ.get("POW_NODE_LOG_DIR"):  # diagnostics: keep the network's output
        with open(os.path.join(os.environ["POW_NODE_LOG_DIR"], f"net_{np_}_{d}.log"), "w") as f:
            f.write(f"wall {time.perf_counter() - t0:.3f} s rc {run.returncode}\n{run.stdout}")
    assert run.returncode == 0, run.stdout[-3000:]
    assert "Error duro" not in run.stdout
    complete = [r for r, entries in run.chains.items() if check_chain(entries, 10, d)]
    assert complete, run.stdout[-3000:]
    assert "Agregué un producido" in run.stdout
    if d <= 5:
        # every rank mined its own block 1 before anyone published one
        assert len(re.findall(r"Agregué un producido con index 1 ", run.stdout)) == np_, run.stdout[-3000:]
        assert RIVAL_BLOCK1.search(run.stdout), run.stdout[-3000:]


@pytest.mark.skipif(not os.path.exists(REF_BIN), reason="reference binary not built")
def test_mixed_with_reference_nodes(tmp_path):
    """2 reference ranks (picosha2, CPU) + 2 GPU ranks in one mpiexec at the
    reference's DEFAULT_DIFFICULTY (9): the reference ranks validate and adopt
    GPU-mined blocks, the GPU ranks validate the reference's."""
    # --serial-init 1: GPU set-up before MPI_Init, so MPI_Init is every rank's
    # start line as in the reference (reference ranks join no start barrier).
    # --idle-below 3: the GPU ranks mine only once the chain holds block 3, so blocks 1-3
    # come from the reference ranks and both directions of adoption are
    # certain (with a timing knob alone, a slow box let the GPU ranks win all
    # 10 blocks in 1 of 2 runs: profiles/r02/verify/protocol_soak_mixed_*.log).
    run = run_network(2, str(tmp_path), difficulty=9, blocks=10, timeout=240, ref_binary=REF_BIN, n_ref=2,
                      extra_args=("--serial-init", "1", "--idle-below", "3"))
    assert run.returncode == 0, run.stdout[-3000:]
    assert "Error duro" not in run.stdout, run.stdout[-3000:]
    # reference ranks 0/1 accepted blocks sent by GPU ranks 2/3
    adopted = re.findall(r"\[(\d)\] Agregado a la lista bloque con index \d+ enviado por (\d)", run.stdout)
    assert any(int(r) < 2 and int(s) >= 2 for r, s in adopted), run.stdout[-3000:]
    # and GPU ranks accepted blocks mined by the reference (validated by K2)
    assert any(int(r) >= 2 and int(s) < 2 for r, s in adopted), run.stdout[-3000:]
    assert [r for r, entries in run.chains.items() if check_chain(entries, 10, 9)]
