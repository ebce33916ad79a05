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


@pytest.fixture(scope="module")
def mpi_exe(tmp_path_factory):
    from mpi_blockchain_amd.build import MPI_HOME, build, mpi_available

    if not mpi_available():
        pytest.skip("no MPI in this image")
    build()
    out = str(tmp_path_factory.mktemp("cm") / "group_mine_mpi")
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    "-I", os.path.join(MPI_HOME, "include"), os.path.join(ROOT, "examples", "group_mine_mpi.c"),
                    "-L", PKG, "-lpow_gpu", f"-Wl,-rpath,{PKG}", os.path.join(MPI_HOME, "lib", "libmpi.so"),
                    # the system libstdc++ first: MPICH's lib dir holds an older one
                    "-Wl,-rpath-link,/lib/x86_64-linux-gnu", f"-Wl,-rpath-link,{os.path.join(MPI_HOME, 'lib')}", "-o", out], check=True)
    return out


def test_group_example_builds(mpi_exe):
    assert os.path.exists(mpi_exe)


@pytest.mark.gpu
def test_group_example_mines(mpi_exe, tmp_path):
    """C + MPI caller of the sharded search: the RCCL id over MPI_Bcast, then
    pow_group_mine; S0 at d = 21 over [0, 2^32): lowest counter 2392323
    (tests/golden/fingerprints_2p32.json)."""
    from mpi_blockchain_amd.node import MPIEXEC, mpi_env

    p = subprocess.run(["timeout", "-k", "10", "240", MPIEXEC, "-np", "1", mpi_exe, "21", "32"],
                       capture_output=True, text=True, cwd=tmp_path, env=mpi_env())
    assert p.returncode == 0, p.stdout + p.stderr
    assert "counter 2392323 " in p.stdout and "agreed and valid" in p.stdout, p.stdout


@pytest.fixture(scope="module")
def board_exe(tmp_path_factory):
    from mpi_blockchain_amd.build import build

    build()
    out = str(tmp_path_factory.mktemp("cb") / "board_two_ctx")
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-D_POSIX_C_SOURCE=200809L", "-I",
                    os.path.join(ROOT, "include"), os.path.join(ROOT, "examples", "board_two_ctx.c"), "-L", PKG,
                    # the test library: POW_GRID_PER_CU=4 (a test-build switch) leaves half the chip to A
                    "-lpow_gpu_test", f"-Wl,-rpath,{PKG}", "-lpthread", "-o", out], check=True)
    return out


def test_board_example_builds(board_exe):
    assert os.path.exists(board_exe)


@pytest.mark.gpu
def test_board_example_stops_peer(board_exe):
    """Two contexts, two host threads, one private stop board, from C: the
    running context stops within 5 ms of the finder's return."""
    p = subprocess.run([board_exe], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, POW_GRID_PER_CU="4"))
    assert p.returncode == 0, p.stdout + p.stderr
    assert "A: rc 1 " in p.stdout and "B: rc 0 " in p.stdout, p.stdout


def _deadline_exe(tmp_path_factory, lib: str) -> str:
    from mpi_blockchain_amd.build import build, build_test_stub

    build()
    build_test_stub()
    out = str(tmp_path_factory.mktemp("cd") / f"group_init_deadline_{lib}")
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-D_POSIX_C_SOURCE=200809L", "-I",
                    os.path.join(ROOT, "include"), os.path.join(ROOT, "examples", "group_init_deadline.c"), "-L", PKG,
                    f"-l{lib}", f"-Wl,-rpath,{PKG}", "-o", out], check=True)
    return out


@pytest.fixture(scope="module")
def deadline_exes(tmp_path_factory):
    return {lib: _deadline_exe(tmp_path_factory, lib) for lib in ("pow_gpu", "pow_gpu_test")}


def test_group_init_deadline_example_builds(deadline_exes):
    assert all(os.path.exists(p) for p in deadline_exes.values())


def _shm_names(prefix: str) -> set:
    return {f for f in os.listdir("/dev/shm") if f.startswith(prefix)} if os.path.isdir("/dev/shm") else set()


@pytest.mark.gpu
@pytest.mark.parametrize("transport", ["rccl_stub", "rccl"])
def test_group_init_deadline(deadline_exes, transport):
    """A rank that never calls pow_group_init: its peer's pow_group_init returns
    POW_ECOMM after the 3 s deadline (non-blocking ncclCommInitRankConfig
    polled by ncclCommGetAsyncError, then ncclCommAbort) instead of waiting
    forever, and the context stays usable (a one-rank group then mines S0 at
    d = 21 to 2392323).  rccl_stub: the test library with the stand-in RCCL;
    rccl: the shipped library with RCCL itself (torch's copy is not loaded
    here: librccl.so.1 from the library path)."""
    from mpi_blockchain_amd.build import STUB_LIB

    env = dict(os.environ)
    if transport == "rccl_stub":
        env["POW_TEST_RCCL_LIB"] = STUB_LIB
    exe = deadline_exes["pow_gpu_test" if transport == "rccl_stub" else "pow_gpu"]
    before = _shm_names("pow_")
    p = subprocess.run(["timeout", "-k", "5", "90", exe, "3000"], capture_output=True, text=True, env=env)
    assert p.returncode == 0, p.stdout + p.stderr[-3000:]
    assert "lonely rank 0 of 2: rc -5 after" in p.stdout and "not every rank joined within 3.000 s" in p.stdout, \
        p.stdout
    assert "one-rank group: counter 2392323," in p.stdout and p.stdout.rstrip().endswith("ok"), p.stdout
    assert _shm_names("pow_") <= before  # the board's and the stand-in's segments are gone
