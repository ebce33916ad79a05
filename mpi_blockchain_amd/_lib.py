"""ctypes binding of ``libpow_gpu.so`` (include/pow_gpu.h, include/pow_tools.h).

There is deliberately NO fallback: if the native library is missing or fails
to load, this raises.  The product path never routes through a CPU
implementation (the CPU checkers live in ``oracle/`` and are test-only).
"""
from __future__ import annotations

import ctypes
import os

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG, "libpow_gpu.so")
# The same library built with -DPOW_TEST_HOOKS (build.py): test and tuning
# switches read from the environment at pow_init.  Only tests load it.
TEST_LIB_PATH = os.path.join(PKG, "libpow_gpu_test.so")

HASH_SIZE = 256
NONCE_SIZE = 10
MSG_BYTES = 270
COUNTER_LIMIT = 62**9

POW_OK, POW_EINVAL, POW_ENOSPC, POW_EHIP, POW_ENODEV, POW_ECOMM = 0, -1, -2, -3, -4, -5
_ERRNAMES = {POW_EINVAL: "POW_EINVAL", POW_ENOSPC: "POW_ENOSPC", POW_EHIP: "POW_EHIP",
             POW_ENODEV: "POW_ENODEV", POW_ECOMM: "POW_ECOMM"}
GROUP_ID_BYTES = 128
BOARD_MAX_SLOTS, BOARD_MAX_TAG = 64, 1023
POW_REDUCE_MIN, POW_REDUCE_MAX, POW_REDUCE_SUM = 0, 1, 2


class PowError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{_ERRNAMES.get(code, code)}: {msg}")
        self.code = code


class Block(ctypes.Structure):
    """``struct Block`` of block.h:17-25 (== ``pow_block``), sizeof 552."""

    _fields_ = [
        ("index", ctypes.c_uint32),
        ("node_owner_number", ctypes.c_uint32),
        ("difficulty", ctypes.c_uint32),
        ("created_at", ctypes.c_uint64),
        ("nonce", ctypes.c_char * NONCE_SIZE),
        ("previous_block_hash", ctypes.c_char * HASH_SIZE),
        ("block_hash", ctypes.c_char * HASH_SIZE),
    ]


# int reduce(void* user, uint64_t* vals, size_t n, int op): pow_group_reduce_fn
REDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t,
                             ctypes.c_int)


class PowStats(ctypes.Structure):
    _fields_ = [("kernel_ms", ctypes.c_double), ("launches", ctypes.c_uint32),
                ("hashes", ctypes.c_uint64)]


class ValuResult(ctypes.Structure):
    """pow_valu_result (include/pow_tools.h)."""

    _fields_ = [("lane_ops_per_s", ctypes.c_double), ("kernel_ms", ctypes.c_double),
                ("clock_hz", ctypes.c_double), ("cycles_per_instr", ctypes.c_double)]


class GroupSearchInfo(ctypes.Structure):
    """pow_group_search_info (include/pow_gpu.h): this rank's part in the
    group's last search."""

    _fields_ = [("board_open", ctypes.c_int), ("board_bound", ctypes.c_int), ("rounds", ctypes.c_uint32),
                ("local_found", ctypes.c_int), ("mine_end_ns", ctypes.c_uint64), ("mine_ms", ctypes.c_double),
                ("allreduce_ms", ctypes.c_double)]


POW_VALU_MIX, POW_VALU_FULL, POW_VALU_HALF = 0, 1, 2
POW_LAUNCH_HIP, POW_LAUNCH_DIRECT = 0, 1

assert ctypes.sizeof(Block) == 552

_libs: dict = {}


def load(test_hooks: bool = False) -> ctypes.CDLL:
    """Load libpow_gpu.so (raises if it is missing — no fallback).
    test_hooks=True: libpow_gpu_test.so, the same code plus the test switches
    (tests only; both may be loaded in one process, each with its own handle)."""
    path = TEST_LIB_PATH if test_hooks else LIB_PATH
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: build it with `python -m mpi_blockchain_amd.build` "
            "(the GPU path has no CPU fallback)")
    # One HIP runtime per process: when PyTorch-ROCm is importable, load it
    # first so this library binds to the same libamdhip64.so.7 (same soname).
    try:
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is optional for the C ABI
        pass
    L = ctypes.CDLL(path)
    P = ctypes.POINTER(Block)
    c_u64p = ctypes.POINTER(ctypes.c_uint64)
    c_sizep = ctypes.POINTER(ctypes.c_size_t)
    sigs = {
        "pow_device_count": ([ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
        "pow_init": ([ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
        "pow_destroy": ([ctypes.c_void_p], None),
        "pow_warmup": ([ctypes.c_void_p], ctypes.c_int),
        "pow_last_error": ([], ctypes.c_char_p),
        "pow_get_stats": ([ctypes.c_void_p, ctypes.POINTER(PowStats)], ctypes.c_int),
        "pow_launch_path": ([ctypes.c_void_p], ctypes.c_int),
        "pow_device_pci_bus_id": ([ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t], ctypes.c_int),
        "pow_device_info": ([ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                             ctypes.c_char_p, ctypes.c_size_t], ctypes.c_int),
        "pow_nonce_from_counter": ([ctypes.c_uint64, ctypes.c_char_p], ctypes.c_int),
        "pow_block_to_bytes": ([P, ctypes.c_char_p], ctypes.c_int),
        "pow_solves_problem": ([ctypes.c_char_p, ctypes.c_uint], ctypes.c_int),
        "pow_hash_blocks": ([ctypes.c_void_p, P, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_char_p],
                            ctypes.c_int),
        "pow_hash_block": ([ctypes.c_void_p, P, ctypes.c_char_p, ctypes.c_char_p], ctypes.c_int),
        "pow_mine": ([ctypes.c_void_p, P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint,
                      ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32, P, c_u64p, c_u64p], ctypes.c_int),
        "pow_mine_any": ([ctypes.c_void_p, P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint,
                          ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32, P, c_u64p, c_u64p], ctypes.c_int),
        "pow_sweep": ([ctypes.c_void_p, P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint,
                       ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t, c_sizep], ctypes.c_int),
        "pow_sweep_device": ([ctypes.c_void_p, P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint,
                              ctypes.c_void_p, ctypes.c_size_t, c_sizep, c_u64p], ctypes.c_int),
        "pow_cancel": ([ctypes.c_void_p, ctypes.c_uint32], ctypes.c_int),
        "pow_dev_alloc": ([ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
        "pow_dev_free": ([ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
        "pow_dev_read": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t], ctypes.c_int),
        "pow_group_partition": ([ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, c_u64p, c_u64p],
                                None),
        "pow_group_unique_id": ([ctypes.c_char_p], ctypes.c_int),
        "pow_group_init": ([ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_char_p,
                            ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
        "pow_group_init_within": ([ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_uint,
                                   ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
        "pow_group_init_custom": ([ctypes.c_void_p, ctypes.c_int, ctypes.c_int, REDUCE_FN, ctypes.c_void_p,
                                   ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
        "pow_group_destroy": ([ctypes.c_void_p], None),
        "pow_group_info": ([ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
        "pow_group_rccl_path": ([ctypes.c_char_p, ctypes.c_size_t], ctypes.c_int),
        "pow_group_last_search": ([ctypes.c_void_p, ctypes.POINTER(GroupSearchInfo)], ctypes.c_int),
        "pow_group_allreduce_u64": ([ctypes.c_void_p, c_u64p, ctypes.c_size_t, ctypes.c_int], ctypes.c_int),
        "pow_group_mine": ([ctypes.c_void_p, P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint,
                            ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32, P, c_u64p, c_u64p], ctypes.c_int),
        "pow_group_mine_any": ([ctypes.c_void_p, P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint,
                                ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32, P, c_u64p, c_u64p], ctypes.c_int),
        "pow_board_open": ([ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
        "pow_board_unlink": ([ctypes.c_char_p], ctypes.c_int),
        "pow_board_close": ([ctypes.c_void_p], None),
        "pow_board_bind": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32], ctypes.c_int),
        "pow_board_post": ([ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint64], ctypes.c_int),
        "pow_board_peek": ([ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, c_u64p], ctypes.c_int),
        "pow_valu_peak": ([ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)],
                          ctypes.c_int),
        "pow_valu_rate": ([ctypes.c_int, ctypes.c_int, ctypes.POINTER(ValuResult)], ctypes.c_int),
        "pow_valu_rate_ctx": ([ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ValuResult)], ctypes.c_int),
    }
    for name, (args, res) in sigs.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _libs[path] = L
    return L


EXPORTS = ("pow_device_count", "pow_init", "pow_warmup", "pow_destroy", "pow_last_error", "pow_get_stats", "pow_launch_path",
           "pow_device_info", "pow_device_pci_bus_id",
           "pow_nonce_from_counter", "pow_block_to_bytes", "pow_solves_problem", "pow_hash_blocks",
           "pow_hash_block", "pow_mine", "pow_mine_any", "pow_cancel", "pow_sweep", "pow_sweep_device", "pow_dev_alloc", "pow_dev_free",
           "pow_dev_read", "pow_valu_peak", "pow_valu_rate", "pow_valu_rate_ctx", "pow_group_partition", "pow_group_unique_id", "pow_group_init",
           "pow_group_init_within",
           "pow_group_init_custom", "pow_group_destroy", "pow_group_info", "pow_group_rccl_path", "pow_group_last_search",
           "pow_group_allreduce_u64", "pow_group_mine", "pow_group_mine_any",
           "pow_board_open", "pow_board_unlink", "pow_board_close", "pow_board_bind", "pow_board_post",
           "pow_board_peek")


def check(rc: int, L: ctypes.CDLL | None = None) -> int:
    """Raise PowError for rc < 0 with the message of the library that failed
    (each loaded library keeps its own pow_last_error)."""
    if rc < 0:
        raise PowError(rc, ((L or load()).pow_last_error() or b"").decode(errors="replace"))
    return rc
