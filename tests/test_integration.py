"""The drop-in, built for real: tests/integration/node_cpp.patch applied to the
REFERENCE's own node.cpp (its proof_of_work trial loop, node.cpp:301-308,
replaced by pow_mine_any; the receive loop, node.cpp:408-409, publishing chain
moves with pow_cancel), compiled with the reference's block.cpp and
blockchain.cpp and linked against libpow_gpu.so — the patch a maintainer
would apply.

CPU: the patch applies to a scratch copy of /root/reference and the result
links (needs /root/reference, i.e. this container).  GPU: the binary that
`make -C oracle ref` built the same way (oracle/_ref/blockchain_dropin; the GPU
box has no /root/reference) mines a 10-block chain at the reference's
DEFAULT_DIFFICULTY in `mpiexec -np 2`, and the chain dumps it writes
(log_chain, node.cpp:40-58) are linked and solving.
"""
import os
import shutil
import subprocess

import pytest

from helpers import check_chain
from mpi_blockchain_amd.build import LIB, MPI_HOME, mpi_available

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
PATCH = os.path.join(ROOT, "tests", "integration", "node_cpp.patch")
DROPIN = os.path.join(ROOT, "oracle", "_ref", "blockchain_dropin")


@pytest.mark.skipif(not os.path.isdir(REF) or not mpi_available() or not os.path.exists(LIB),
                    reason="needs /root/reference, MPI and libpow_gpu.so")
def test_patch_applies_and_links(tmp_path):
    src = tmp_path / "ref"
    src.mkdir()
    for f in os.listdir(REF):
        if f.endswith((".cpp", ".h")):
            shutil.copy(os.path.join(REF, f), src / f)
    subprocess.run(["patch", "-s", "-d", str(src), "-p1", "-i", PATCH], check=True)
    node = (src / "node.cpp").read_text()
    body = node[node.index("void* proof_of_work"):node.index("int send_blockchain")]
    # the trial loop is gone from proof_of_work; the GPU round and the unchanged success tail are there
    assert "gen_random_nonce(block" not in body and "solves_problem(hash" not in body
    assert "pow_mine_any(" in body and "send_block_to_everyone(*last_block_in_chain)" in body
    assert node.count("pow_cancel(") == 2  # arm once, then on every chain move
    # only node.cpp changes
    for f in ("block.cpp", "blockchain.cpp", "block.h", "node.h"):
        assert (src / f).read_bytes() == open(os.path.join(REF, f), "rb").read()
    exe = tmp_path / "blockchain"
    subprocess.run(["g++", "-std=c++11", "-pthread", "-g", f"-I{src}", f"-I{ROOT}/include",
                    f"-I{MPI_HOME}/include", "-o", str(exe), str(src / "node.cpp"), str(src / "block.cpp"),
                    str(src / "blockchain.cpp"), f"-L{os.path.dirname(LIB)}", "-lpow_gpu",
                    f"-Wl,-rpath,{os.path.dirname(LIB)}", os.path.join(MPI_HOME, "lib", "libmpi.so"),
                    f"-Wl,-rpath-link,{os.path.join(MPI_HOME, 'lib')}"], check=True, capture_output=True)
    undef = subprocess.run(["nm", "-u", str(exe)], capture_output=True, text=True, check=True).stdout
    for sym in ("pow_init", "pow_warmup", "pow_mine_any", "pow_cancel", "pow_device_count"):
        assert sym in undef


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(DROPIN) or not mpi_available(), reason="drop-in binary not built")
def test_dropin_mines_chain(tmp_path):
    from mpi_blockchain_amd.node import MPIEXEC, mpi_env, parse_chain_dump

    # the reference's main() runs `rm *.out` in its cwd (blockchain.cpp:31): a scratch dir
    p = subprocess.run(["timeout", "-k", "10", "180", MPIEXEC, "-np", "2", DROPIN], cwd=tmp_path,
                       env=mpi_env(), capture_output=True, text=True)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-3000:]
    assert "Error duro" not in out and "pow_mine_any:" not in out, out[-3000:]
    assert "Agregué un producido" in out
    chains = {r: parse_chain_dump((tmp_path / f"{r}.out").read_text())
              for r in range(2) if (tmp_path / f"{r}.out").exists()}
    complete = [r for r, entries in chains.items() if check_chain(entries, 10, 9)]  # BLOCKS_TO_MINE, DEFAULT_DIFFICULTY
    assert complete, out[-3000:]
