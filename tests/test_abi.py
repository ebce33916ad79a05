"""The C-ABI library (libpow_gpu.so): it loads, exports every entry point the
headers declare, and its host-side helpers (no GPU work) reproduce the
reference's serializer / nonce alphabet / difficulty test.  CPU only."""
import ctypes
import os
import random
import re

import pytest

from mpi_blockchain_amd import _lib
from mpi_blockchain_amd.block import (block_to_str, gen_random_nonce, make_block, nonce_from_counter,
                                      solves_problem)
from oracle.oracle import py_solves_problem

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    names = set()
    for h in ("pow_gpu.h", "pow_tools.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"^\s*(?:const\s+)?\w[\w\s\*]*?\b(pow_\w+)\s*\(", src, flags=re.M))
    return names


def test_headers_declare_expected_entry_points():
    names = header_functions()
    for f in ("pow_init", "pow_destroy", "pow_hash_block", "pow_mine", "pow_sweep", "pow_nonce_from_counter"):
        assert f in names
    assert names == set(_lib.EXPORTS), names ^ set(_lib.EXPORTS)


def test_library_exports_all_symbols():
    L = _lib.load()
    for name in header_functions():
        assert hasattr(L, name), name


HOOKS = (b"POW_FAULT_INJECT", b"POW_FORCE_FULL", b"POW_LAT_MAX", b"POW_LAT_WPS", b"POW_GRID_PER_CU", b"POW_TEST_SENTINEL_IDLE",
         b"POW_TEST_RCCL_LIB", b"POW_AQL", b"POW_AQL_EXP", b"POW_AQL_STALL_US", b"POW_WATCHDOG_MS", b"POW_TEST_STALL_US")


def test_shipped_library_has_no_test_hooks():
    """The test and tuning switches (fault injection, forced kernel variants,
    launch geometry, the stand-in RCCL) exist only in libpow_gpu_test.so,
    built from the same objects plus -DPOW_TEST_HOOKS (build.py); the shipped
    libpow_gpu.so reads no such variable.  Both export the same ABI."""
    shipped = open(_lib.LIB_PATH, "rb").read()
    test = open(_lib.TEST_LIB_PATH, "rb").read()
    assert [h for h in HOOKS if h in shipped] == []
    assert all(h in test for h in HOOKS)
    T = _lib.load(test_hooks=True)
    assert T is not _lib.load()
    for name in header_functions():
        assert hasattr(T, name), name


def test_shipped_library_launches_through_hip_only():
    """Round 5: direct AQL dispatch (pow_aql.cpp) is linked into the test
    library only.  The shipped library neither links the HSA runtime nor holds
    the dispatcher or the offload-bundle reader: every kernel goes out through
    hipLaunchKernel."""
    shipped = open(_lib.LIB_PATH, "rb").read()
    test = open(_lib.TEST_LIB_PATH, "rb").read()
    for marker in (b"libhsa-runtime64", b"pow_aql_open"):
        assert marker not in shipped, marker
    assert b"libhsa-runtime64" in test and b"pow_aql_open" in test
    # the watchdog's diagnostics are in both
    for lib in (shipped, test):
        assert b"watchdog: no result after" in lib and b"watchdog: not complete after" in lib


def test_block_layout():
    assert ctypes.sizeof(_lib.Block) == 552
    assert _lib.Block.nonce.offset == 24 and _lib.Block.block_hash.offset == 290


def test_nonce_from_counter(golden):
    for e in golden["digests"]:
        assert nonce_from_counter(e["counter"]) == e["nonce"].encode() + b"\0"
    with pytest.raises(_lib.PowError):
        nonce_from_counter(62**9)


def test_block_to_str(golden, templates):
    from helpers import block_from_template, with_nonce

    for name, hx in golden["messages"].items():
        b = with_nonce(block_from_template(templates[name]), nonce_from_counter(0))
        assert block_to_str(b).hex() == hx


def test_solves_problem_matches_reference_semantics():
    rng = random.Random(5)
    alphabet = "0123456789abcdefABCDEFqz"
    for _ in range(3000):
        h = "".join(rng.choice(alphabet) for _ in range(rng.randrange(0, 70)))
        d = rng.randrange(0, 300)
        assert solves_problem(h, d) == py_solves_problem(h, d), (h, d)


def test_gen_random_nonce_alphabet():
    rng = random.Random(1)
    for _ in range(50):
        n = gen_random_nonce(rng)
        assert len(n) == 10 and n[9] == 0 and n[:9].decode().isalnum()


def test_make_block_truncation_fields():
    b = make_block(300, 7, 9, 0x1000000FF, b"Z" * 64)
    assert block_to_str(b)[:4] == bytes([0x2C, 7, 9, 0xFF])


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU is present")
def test_init_fails_cleanly_without_gpu():
    L = _lib.load()
    ctx = ctypes.c_void_p()
    rc = L.pow_init(0, ctypes.byref(ctx))
    assert rc < 0 and not ctx
    assert L.pow_last_error()


def test_null_arguments_rejected():
    L = _lib.load()
    b = make_block()
    out = _lib.Block()
    assert L.pow_mine(None, ctypes.byref(b), 0, 1, 9, None, 0, ctypes.byref(out), None, None) == _lib.POW_EINVAL
    n = ctypes.c_size_t()
    assert L.pow_sweep(None, ctypes.byref(b), 0, 1, 9, None, 0, ctypes.byref(n)) == _lib.POW_EINVAL
    assert L.pow_nonce_from_counter(0, None) == _lib.POW_EINVAL
    assert L.pow_launch_path(None) == _lib.POW_EINVAL


def test_sweep_cap_limit():
    """pow_sweep sorts its list on the device (hipCUB takes a signed 32-bit
    count): a cap of 2^31 or more is rejected before any HIP call, and the
    Python mirror's default cap never reaches it (2^32 window at d <= 1)."""
    L = _lib.load()
    b = make_block()
    n = ctypes.c_size_t()
    for cap in (1 << 31, (1 << 32) - 1, 1 << 40):
        assert L.pow_sweep(None, ctypes.byref(b), 0, 1 << 32, 0, None, cap, ctypes.byref(n)) == _lib.POW_EINVAL
        assert b"2^31-1" in L.pow_last_error()
    import inspect

    from mpi_blockchain_amd.miner import GpuMiner

    src = inspect.getsource(GpuMiner.sweep)
    assert "(1 << 31) - 1" in src
