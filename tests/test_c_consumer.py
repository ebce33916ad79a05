"""A plain-C program against include/pow_gpu.h: it compiles and links on CPU,
and on the GPU it mines and re-validates a 10-block chain."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mpi_blockchain_amd")


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    from mpi_blockchain_amd.build import build

    build()
    out = str(tmp_path_factory.mktemp("c") / "mine_chain")
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "examples", "mine_chain.c"), "-L", PKG, "-lpow_gpu",
                    f"-Wl,-rpath,{PKG}", "-o", out], check=True)
    return out


def test_c_consumer_builds(exe):
    assert os.path.exists(exe)


@pytest.mark.gpu
def test_c_consumer_mines_valid_chain(exe):
    p = subprocess.run([exe, "10", "12"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    assert "chain of 10 blocks at difficulty 12: valid" in p.stdout
