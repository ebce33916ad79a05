"""The protocol node's build (CPU only): bin/pow_node behaves only as
node.cpp does; the race-shaping switches the protocol tests use exist only in
bin/pow_node_test (-DPOW_NODE_TEST_KNOBS)."""
import subprocess

import pytest

from mpi_blockchain_amd.build import build_node, mpi_available
from mpi_blockchain_amd.node import mpi_env

pytestmark = pytest.mark.skipif(not mpi_available(), reason="no MPI in this image")

KNOBS = ("--hold-first", "--idle-below", "--private-lead", "--pause-us", "--pause-ms", "--winner-pause-us",
         "--lead-barrier", "--recv-delay-rank", "--recv-delay-us")


@pytest.mark.parametrize("knob", KNOBS)
def test_product_node_refuses_test_knobs(tmp_path, knob):
    # options are parsed before MPI_Init and before any GPU call
    p = subprocess.run([build_node(), knob, "1"], capture_output=True, text=True, timeout=60, cwd=str(tmp_path),
                       env=mpi_env())
    assert p.returncode == 2 and "pow_node_test" in p.stderr, (p.returncode, p.stderr)


def test_test_node_knows_them():
    """Every knob string is compiled into the test build only."""
    prod = open(build_node(), "rb").read()
    test = open(build_node(test=True), "rb").read()
    for k in KNOBS:
        assert k.encode() in test and k.encode() not in prod, k


def _chain(n: int, rng):
    """A synthetic linked chain, tip first (block 1's prev is empty, node.cpp:369)."""
    from mpi_blockchain_amd.node import ChainEntry

    hashes = ["".join(rng.choice("0123456789abcdef") for _ in range(64)) for _ in range(n)]
    return [ChainEntry(n - i, rng.randrange(1 << 32), hashes[n - i - 2] if n - i - 2 >= 0 else "", hashes[n - i - 1])
            for i in range(n)]


@pytest.mark.parametrize("n", [1, 10, 37])
def test_chain_dump_matches_reference(tmp_path, n):
    """pow_node's termination dump (log_msg + log_chain,
    run through pow_node_test --log-chain-stdin: the same member functions,
    no MPI, no GPU) is byte-identical to what the reference's own node.cpp
    writes for the same chain (oracle/_ref/ref_log_chain), and parses back
    into the chain (mpi_blockchain_amd.node.parse_chain_dump)."""
    import os
    import random

    from helpers import REF_LOG_CHAIN, reference_dump
    from mpi_blockchain_amd.node import parse_chain_dump

    if not os.path.exists(REF_LOG_CHAIN):
        pytest.skip("oracle/_ref/ref_log_chain not built (needs /root/reference)")
    chain = _chain(n, random.Random(n))
    tsv = "".join(f"{e.index}\t{e.owner}\t{e.prev}\t{e.hash}\n" for e in chain)
    p = subprocess.run([build_node(test=True), "--log-chain-stdin", "5"], input=tsv.encode(), cwd=str(tmp_path),
                       env=mpi_env(), capture_output=True, timeout=60)
    assert p.returncode == 0, p.stderr
    ours = (tmp_path / "5.out").read_bytes()
    assert ours == reference_dump(chain, 5)
    assert parse_chain_dump(ours.decode()) == chain
