"""The protocol node's build (CPU only): bin/pow_node behaves only as
node.cpp does; the race-shaping switches the protocol tests use exist only in
bin/pow_node_test (-DPOW_NODE_TEST_KNOBS)."""
import subprocess

import pytest

from mpi_blockchain_amd.build import build_node, mpi_available
from mpi_blockchain_amd.node import mpi_env

pytestmark = pytest.mark.skipif(not mpi_available(), reason="no MPI in this image")

KNOBS = ("--hold-first", "--idle-below", "--private-lead", "--pause-us", "--pause-ms", "--winner-pause-us")


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
