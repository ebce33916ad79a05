"""Protocol runs (BASELINE config 5, scaled to one GPU): MPI networks of
``pow_node`` ranks mining on the GPU through pow_mine, and a mixed network with
the REFERENCE's own binary (oracle/_ref/blockchain_ref, built from
/root/reference) — the reference's picosha2 validation (valid_new_block,
block.cpp:13-25) accepting GPU-mined blocks, and pow_node accepting the
reference's, is the wire-level parity check.  Every
chain dump a run leaves (<rank>.out) is compared byte for byte with what the
reference's own log_msg + log_chain (node.cpp:40-68) write for that chain
(oracle/_ref/ref_log_chain).
"""
import os
import re
import time

import pytest

from helpers import REF_LOG_CHAIN, check_chain, reference_dump
from mpi_blockchain_amd.build import mpi_available
from mpi_blockchain_amd.node import chain_status, run_network

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not mpi_available(), reason="no MPI in this image")]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_BIN = os.path.join(ROOT, "oracle", "_ref", "blockchain_ref")


FORK_MSGS = ("Perdí la carrera", "Conflicto suave", "TAG_CHAIN_HASH")


def keep_log(run, name, wall=None):
    """Diagnostics: with POW_NODE_LOG_DIR set (tools/gpu_pass.sh sets it under
    gpurun_out/), every network's whole output is kept, so a failing pass's
    log survives the re-runs that follow it."""
    d = os.environ.get("POW_NODE_LOG_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, f"{name}.log"), "w") as f:
            f.write(f"rc {run.returncode}" + (f" wall {wall:.3f} s" if wall is not None else "") + f"\n{run.stdout}")
# A rival block 1 received while this rank's chain is at index 1 (node.cpp:235)
# or already past it (node.cpp:242): the fork --hold-first forces.
RIVAL_BLOCK1 = re.compile(r"Conflicto suave: (Conflicto de branch \(1\)|Descarto el bloque \(1 vs \d+\))")


@pytest.mark.parametrize("np_, d", [(4, 9), (6, 5), (8, 5)])  # protocol smoke at d = 5, -np 8
def test_gpu_network(tmp_path, np_, d):
    # Every rank starts mining at the same start line (the MPI_Barrier after
    # GPU set-up in pow_node's main).  At d = 5 the fork is forced rather
    # than left to timing: --hold-first makes every rank mine block 1 and
    # publish it only after a barrier, so every rank receives rival blocks 1.
    # --winner-pause-us 3000: a block's finder waits 3 ms before mining the
    # next, so the losers' chain migrations finish before the finder (~20 us
    # per block at d = 5) completes the chain and MPI_Abort ends the job.
    extra = ("--hold-first", "1", "--winner-pause-us", "3000") if d <= 5 else ()
    t0 = time.perf_counter()
    run = run_network(np_, str(tmp_path), difficulty=d, blocks=10, timeout=240, extra_args=extra)
    keep_log(run, f"net_{np_}_{d}", time.perf_counter() - t0)
    assert run.returncode == 0, run.stdout[-3000:]
    assert "Error duro" not in run.stdout
    complete = [r for r, entries in run.chains.items() if check_chain(entries, 10, d)]
    assert complete, run.stdout[-3000:]
    assert "Agregué un producido" in run.stdout
    assert_dumps_match_reference(run)
    if d <= 5:
        # every rank mined its own block 1 before anyone published one
        assert len(re.findall(r"Agregué un producido con index 1 ", run.stdout)) == np_, run.stdout[-3000:]
        assert RIVAL_BLOCK1.search(run.stdout), run.stdout[-3000:]
        # ... and a chain migration (verificar_y_migrar_cadena, node.cpp:152-191)
        # that requested, checked and spliced a peer's branch
        assert MIGRATED.search(run.stdout), run.stdout[-3000:]


def assert_dumps_match_reference(run):
    """Every complete chain dump (<rank>.out) the run left is byte-identical to
    the reference's own dump of the same chain (log_msg("Terminé con la
    siguiente cadena") + log_chain(""), node.cpp:286-289 -> 40-68).  A rank
    that reached the end too but was killed by the first finisher's MPI_Abort
    (node.cpp:330) while writing leaves a cut dump: it must be a byte prefix of
    a complete one's reference dump."""
    if not os.path.exists(REF_LOG_CHAIN):
        pytest.skip("oracle/_ref/ref_log_chain not built")
    refs = {}
    for r, raw in run.dumps.items():
        if chain_status(run.chains[r], 10, 0)[1]:
            refs[r] = reference_dump(run.chains[r], r)
            assert raw == refs[r], (r, raw[:400])
    assert refs, run.stdout[-3000:]
    for r, raw in run.dumps.items():
        if r not in refs:
            assert any(ref.startswith(raw) for ref in refs.values()), (r, raw[:400])


@pytest.mark.skipif(not os.path.exists(REF_BIN), reason="reference binary not built")
def test_mixed_with_reference_nodes(tmp_path):
    """2 reference ranks (the reference's own binary: picosha2 on the CPU) + 2
    pow_node ranks in one mpiexec at the reference's DEFAULT_DIFFICULTY (9).
    The reference ranks receive pow_node's MPI_BLOCKs (block.cpp:99-120: 542-B
    payload, 552-B extent), validate them with picosha2 (valid_new_block,
    block.cpp:13-25; validate_block_for_chain, node.cpp:194-257) and adopt
    them; the pow_node ranks validate (K2') and adopt the reference's.  One
    complete consistent chain; its dump is the reference's format byte for
    byte."""
    # --serial-init 1: GPU set-up before MPI_Init, so MPI_Init is every rank's
    # start line as in the reference (reference ranks join no start barrier).
    # --idle-below 3 (pow_node_test): the GPU ranks mine only once the chain
    # holds block 3, so blocks 1-3 come from the reference ranks and both
    # directions of adoption are certain (with a timing knob alone, a slow box
    # let the GPU ranks win all 10 blocks in 1 of 2 runs:
    # profiles/r02/verify/protocol_soak_mixed_*.log).
    run = run_network(2, str(tmp_path), difficulty=9, blocks=10, timeout=240, ref_binary=REF_BIN, n_ref=2,
                      extra_args=("--serial-init", "1", "--idle-below", "3"))
    keep_log(run, "mixed_2ref_2gpu")
    out = run.stdout
    assert run.returncode == 0, out[-3000:]
    assert "Error duro" not in out, out[-3000:]
    adopted = [(int(r), int(s)) for r, s in
               re.findall(r"\[(\d)\] Agregado a la lista bloque con index \d+ enviado por (\d)", out)]
    # reference ranks 0/1 accepted blocks mined by pow_node ranks 2/3 ...
    assert any(r < 2 <= s for r, s in adopted), out[-3000:]
    # ... and pow_node ranks accepted blocks mined by the reference
    assert any(s < 2 <= r for r, s in adopted), out[-3000:]
    st = {r: chain_status(c, 10, 9) for r, c in run.chains.items()}
    assert st and all(ok for ok, _ in st.values()) and any(done for _, done in st.values()), (st, out[-3000:])
    # the chain holds blocks of both kinds of miner
    owners = {e.owner for c in run.chains.values() for e in c}
    assert owners & {0, 1} and owners & {2, 3}, owners
    assert_dumps_match_reference(run)


# node.cpp:176: the splice of a checked chain; i >= 0 is the common ancestor's slot
MIGRATED = re.compile(r"\[(\d+)\]: find = (\d+) \| received_blockchain_checks = 1")


@pytest.mark.parametrize("np_", [2, 4])
def test_mutual_chain_request(tmp_path, np_):
    """the reference blocks in MPI_Recv(TAG_CHAIN_RESPONSE)
    while holding the mutex its receive loop needs (node.cpp:155-161,
    404-405), so two ranks that request each other's chains deadlock.  With
    --private-lead 3 (pow_node_test) every rank mines blocks 1..3 on a private
    branch and all publish their tips at once: every rank is 3 behind ("Perdí
    la carrera por varios"), asks the tip's owner for its chain while that
    owner asks it, serves the owner's TAG_CHAIN_HASH inside its own wait,
    receives the chain, checks it and splices it in (find = 2: block 1 is the
    common point with genesis).  No rank mines block 4 before every rank has
    migrated (pow_node_test's second barrier, round 5), so the first rank to
    finish cannot abort the job before a slower rank has logged its migration.
    The network then finishes its 10 blocks."""
    run = run_network(np_, str(tmp_path), difficulty=9, blocks=10, timeout=120, extra_args=("--private-lead", "3"))
    keep_log(run, f"mutual_{np_}")
    out = run.stdout
    assert run.returncode == 0, out[-3000:]
    assert "Error duro" not in out, out[-3000:]
    for r in range(np_):
        assert len(re.findall(rf"\[{r}\] Bloque privado con index \d ", out)) == 3, out[-3000:]
        assert f"[{r}] Perdí la carrera por varios contra" in out, out[-3000:]
        assert f"[{r}]: find = 2 | received_blockchain_checks = 1" in out, out[-3000:]
    served = re.findall(r"\[(\d+)\] TAG_CHAIN_HASH de (\d+) atendido mientras espero la cadena de (\d+)", out)
    if np_ == 2:  # each rank served its peer's request while waiting for that same peer's chain
        assert {(int(a), int(b), int(c)) for a, b, c in served} >= {(0, 1, 1), (1, 0, 0)}, out[-3000:]
    else:
        assert served, out[-3000:]
    # the rank that completes the chain dumps it and aborts the job (node.cpp:286-290, 330)
    st = [chain_status(c, 10, 9) for c in run.chains.values()]
    assert st and all(ok for ok, _ in st) and any(done for _, done in st), out[-3000:]
    assert_dumps_match_reference(run)


def _silent_after_tip(out: str, r: int) -> bool:
    """Round 4's failure shape: rank r mined its private branch but never
    logged losing the race (node.cpp:249-253), i.e. never validated a tip."""
    return len(re.findall(rf"\[{r}\] Bloque privado con index \d ", out)) == 3 and \
        f"[{r}] Perdí la carrera por varios contra" not in out


def test_private_lead_termination_race_reproduced(tmp_path):
    """Round 4's one failed pass, reproduced on purpose and closed (DESIGN.md
    §4, "Direct dispatch, round 5").  Rank 3's receive thread is made slow
    (pow_node_test --recv-delay-rank 3 --recv-delay-us 150000: it sleeps
    150 ms after the tips' barrier, before its first validation).
    * Without the miners' barrier after every migration (--lead-barrier 0,
      round 4's test shape), ranks that migrated mine blocks 4..10 in a few ms
      and the finisher's MPI_Abort (node.cpp:330) ends the job while rank 3 is
      still asleep: rc 0, and rank 3 never logs its lost race, the exact shape
      of the failure, with no GPU launch involved.
    * With the barrier (the default) the same slow rank holds every miner
      until it has migrated, and every rank logs its migration."""
    runs = []
    for k in range(4):
        (tmp_path / f"old{k}").mkdir()
        run = run_network(4, str(tmp_path / f"old{k}"), difficulty=9, blocks=10, timeout=120,
                          extra_args=("--private-lead", "3", "--lead-barrier", "0",
                                      "--recv-delay-rank", "3", "--recv-delay-us", "150000"))
        keep_log(run, f"termination_race_old_shape_{k}")
        assert run.returncode == 0, run.stdout[-3000:]
        runs.append(_silent_after_tip(run.stdout, 3))
    print(f"round-4 shape, slow rank 3: silent in {sum(runs)} of {len(runs)} networks")
    assert any(runs), "the termination race did not show"
    for k in range(2):
        (tmp_path / f"new{k}").mkdir()
        run = run_network(4, str(tmp_path / f"new{k}"), difficulty=9, blocks=10, timeout=120,
                          extra_args=("--private-lead", "3", "--recv-delay-rank", "3", "--recv-delay-us", "150000"))
        keep_log(run, f"termination_race_fixed_{k}")
        out = run.stdout
        assert run.returncode == 0, out[-3000:]
        for r in range(4):
            assert f"[{r}] Perdí la carrera por varios contra" in out, (r, out[-3000:])
            assert f"[{r}]: find = 2 | received_blockchain_checks = 1" in out, (r, out[-3000:])


def test_node_reports_placement(tmp_path):
    """Every pow_node rank says which GPU it mines on: one `pow_node device`
    line with the HIP device, the PCI address and the launcher variable that
    chose it.  Under MPICH's mpiexec that is MPI_LOCALRANKID;
    without it the node falls back to PMI_RANK (the global rank: the same on
    one node).  MPICH cannot run a rank without PMI_RANK, so the no-variable
    warning is covered by the CPU test of bench.node_placement."""
    import subprocess
    import sys

    sys.path.insert(0, ROOT)
    import bench
    from mpi_blockchain_amd.build import build_node
    from mpi_blockchain_amd.node import MPIEXEC, mpi_env

    node = build_node()
    strip = ["env", "-u", "MPI_LOCALRANKID", "-u", "OMPI_COMM_WORLD_LOCAL_RANK", "-u", "LOCAL_RANK"]
    for name, prefix, want in (("launcher", [], "MPI_LOCALRANKID"), ("pmi_rank", strip, "PMI_RANK")):
        d = tmp_path / name
        d.mkdir()
        p = subprocess.run(["timeout", "-k", "10", "120", MPIEXEC, "-np", "2", *prefix, node, "--difficulty", "9"],
                           cwd=d, env=mpi_env(), capture_output=True, text=True)
        assert p.returncode == 0, (name, p.stdout[-2000:], p.stderr[-2000:])
        pl = bench.node_placement(p.stdout + p.stderr, 2, rehearsal=True)
        assert pl["ok"] and pl["all_ranks_reported"] and pl["no_local_rank_warnings"] == [], (name, pl)
        assert [x["rank"] for x in pl["devices"]] == [0, 1] and [x["local_rank"] for x in pl["devices"]] == [0, 1], pl
        assert [x["local_rank_from"] for x in pl["devices"]] == [want] * 2, (name, pl)
        assert all(re.fullmatch(r"[0-9a-f]{4}:[0-9a-f]{2}:[0-9a-f]{2}\.[0-9a-f]", x["pci"], re.I)
                   for x in pl["devices"]), pl
