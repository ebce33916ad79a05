"""GPU miner: the proof_of_work hot path (node.cpp:278-332) on one MI355X.

:class:`GpuMiner` owns one ``pow_ctx`` (one GPU, one HIP stream).  Like the
reference's mining pthread it is driven by exactly one thread; other threads
may only bump the cancel word (:meth:`GpuMiner.cancel`).
"""
from __future__ import annotations

import ctypes
import time
from dataclasses import dataclass

import numpy as np

from ._lib import HASH_SIZE, Block, PowStats, check, load
from .block import DEFAULT_DIFFICULTY, field, nonce_from_counter


@dataclass
class MineResult:
    block: Block          # the solved block (nonce + block_hash filled)
    counter: int          # counter whose nonce solved it (lowest in range)
    hashes: int           # trials issued
    kernel_ms: float      # GPU time of the call


def refresh_template(last: Block, rank: int, difficulty: int = DEFAULT_DIFFICULTY,
                     now: int | None = None) -> Block:
    """node.cpp:292-299: copy the last block, index+1, owner = rank,
    difficulty = DEFAULT_DIFFICULTY, created_at = time(NULL), and
    memcpy(prev, last.block_hash, 256) — all 256 bytes (trap T5)."""
    b = Block()
    ctypes.pointer(b)[0] = last
    b.index = (last.index + 1) & 0xFFFFFFFF
    b.node_owner_number = rank & 0xFFFFFFFF
    b.difficulty = difficulty & 0xFFFFFFFF
    b.created_at = int(time.time()) if now is None else now
    ctypes.memmove(ctypes.addressof(b) + Block.previous_block_hash.offset,
                   ctypes.addressof(last) + Block.block_hash.offset, HASH_SIZE)
    return b


class GpuMiner:
    def __init__(self, device: int = 0, test_hooks: bool = False):
        """test_hooks=True: a context of libpow_gpu_test.so, which reads the
        test switches (POW_FORCE_FULL, POW_LAT_MAX, POW_GRID_PER_CU, ...) from
        the environment at pow_init; tests only."""
        self.L = load(test_hooks)
        self.ctx = ctypes.c_void_p()
        check(self.L.pow_init(device, ctypes.byref(self.ctx)), self.L)
        self.device = device
        self._cancel = ctypes.c_uint32(0)

    def warmup(self) -> None:
        """Load every kernel now (HIP loads code objects at first launch)."""
        check(self.L.pow_warmup(self.ctx), self.L)

    # ---- lifecycle ----
    def close(self) -> None:
        if self.ctx:
            self.L.pow_destroy(self.ctx)
            self.ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # ---- info ----
    def device_info(self) -> dict:
        cu, clk = ctypes.c_int(), ctypes.c_int()
        name = ctypes.create_string_buffer(256)
        check(self.L.pow_device_info(self.ctx, ctypes.byref(cu), ctypes.byref(clk), name, 256), self.L)
        return {"cu_count": cu.value, "clock_khz": clk.value, "name": name.value.decode()}

    def pci_bus_id(self) -> str:
        """The GPU as "domain:bus:device.function" (pow_device_pci_bus_id)."""
        buf = ctypes.create_string_buffer(64)
        check(self.L.pow_device_pci_bus_id(self.ctx, buf, len(buf)), self.L)
        return buf.value.decode()

    def launch_path(self) -> str:
        """How the latency-bound launches go out (pow_launch_path): "hip"
        (hipLaunchKernel; the shipped library's only path) or "direct" (AQL
        packets into the process's dispatch queue: test library with
        POW_AQL=1)."""
        return "direct" if check(self.L.pow_launch_path(self.ctx), self.L) == 1 else "hip"

    def stats(self) -> dict:
        s = PowStats()
        check(self.L.pow_get_stats(self.ctx, ctypes.byref(s)), self.L)
        return {"kernel_ms": s.kernel_ms, "launches": s.launches, "hashes": s.hashes}

    # ---- block_to_hash (block.cpp:74-77) ----
    def hash_blocks(self, blocks) -> list[str]:
        n = len(blocks)
        if n == 0:
            return []
        arr = (Block * n)(*blocks)
        hx = ctypes.create_string_buffer(65 * n)
        check(self.L.pow_hash_blocks(self.ctx, arr, n, None, hx), self.L)
        raw = hx.raw
        return [raw[65 * i: 65 * i + 64].decode() for i in range(n)]

    def block_to_hash(self, b: Block) -> str:
        return self.hash_blocks([b])[0]

    def digest(self, b: Block) -> bytes:
        dg = ctypes.create_string_buffer(32)
        check(self.L.pow_hash_block(self.ctx, ctypes.byref(b), dg, None), self.L)
        return dg.raw

    # ---- mining ----
    def cancel(self) -> None:
        """Called from another thread (the receive loop) when the chain moved:
        bumps the cancel word and publishes it to the GPU (pow_cancel), so a
        running mine call stops within one inner step, not at its next
        sub-round."""
        self._cancel.value = (self._cancel.value + 1) & 0xFFFFFFFF
        check(self.L.pow_cancel(self.ctx, self._cancel.value), self.L)

    @property
    def epoch(self) -> int:
        return self._cancel.value

    def bind_board(self, board: "StopBoard | None", slot: int = 0, tag: int = 1) -> None:
        """Join a search shared with other GPUs / contexts (pow_board_bind):
        this miner's hits go to `slot` of `board`, and its mine calls stop as
        soon as a peer slot of the same `tag` makes its remaining counters
        moot.  board=None unbinds."""
        check(self.L.pow_board_bind(self.ctx, board.ptr if board is not None else None, slot, tag), self.L)

    def mine(self, tmpl: Block, start: int = 0, count: int = 1 << 40, difficulty: int = DEFAULT_DIFFICULTY,
             epoch: int | None = None, any_solution: bool = False) -> MineResult | None:
        """Lowest solving counter in [start, start+count) (pow_mine), or the
        first one found (pow_mine_any, lowest latency); None if none / cancelled."""
        out = Block()
        ctr, hashes = ctypes.c_uint64(), ctypes.c_uint64()
        ep = self._cancel.value if epoch is None else epoch
        fn = self.L.pow_mine_any if any_solution else self.L.pow_mine
        rc = check(fn(self.ctx, ctypes.byref(tmpl), start, count, difficulty,
                      ctypes.byref(self._cancel), ep, ctypes.byref(out),
                      ctypes.byref(ctr), ctypes.byref(hashes)), self.L)
        if rc == 0:
            return None
        return MineResult(out, ctr.value, hashes.value, self.stats()["kernel_ms"])

    def sweep(self, tmpl: Block, start: int, count: int, difficulty: int, cap: int | None = None) -> np.ndarray:
        """Ascending (counter - start) of every solving counter (count <= 2^32)."""
        if cap is None:  # pow_sweep sorts on the device: at most 2^31 - 1 entries
            cap = int(min(count, (count >> min(difficulty, 63)) * 2 + 4096, (1 << 31) - 1))
        out = np.zeros(max(cap, 1), dtype=np.uint32)
        n = ctypes.c_size_t()
        check(self.L.pow_sweep(self.ctx, ctypes.byref(tmpl), start, count, difficulty,
                               out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), cap, ctypes.byref(n)), self.L)
        return out[: n.value]  # a view: copying 33.6 MB (a 2^32 window at d = 9) again costs ~3 ms

    def sweep_count(self, tmpl: Block, start: int, count: int, difficulty: int,
                    dev_out=None, cap: int = 0) -> tuple[int, int | None]:
        """Count + lowest solving counter; the list (if any) stays on the GPU."""
        n, mn = ctypes.c_size_t(), ctypes.c_uint64()
        ptr = dev_out.ptr if isinstance(dev_out, DeviceBuffer) else dev_out
        check(self.L.pow_sweep_device(self.ctx, ctypes.byref(tmpl), start, count, difficulty,
                                      ptr if ptr else None, cap,
                                      ctypes.byref(n), ctypes.byref(mn)), self.L)
        return n.value, (None if mn.value == 0xFFFFFFFFFFFFFFFF else mn.value)


class StopBoard:
    """Cross-GPU stop board (include/pow_gpu.h): one slot per rank of a shared
    search, in host memory every GPU of the node maps.  name=None: private to
    this process; name="/x": POSIX shared memory, shared by every process of
    the node that opens it."""

    NONE = None

    def __init__(self, nslots: int, name: str | None = None, test_hooks: bool = False):
        self.L = load(test_hooks)
        self.name = name
        self.ptr = ctypes.c_void_p()
        check(self.L.pow_board_open(name.encode() if name else None, nslots, ctypes.byref(self.ptr)), self.L)

    def post(self, slot: int, tag: int, counter: int | None) -> None:
        check(self.L.pow_board_post(self.ptr, slot, tag, 0xFFFFFFFFFFFFFFFF if counter is None else counter), self.L)

    def peek(self, except_slot: int, tag: int) -> int | None:
        v = ctypes.c_uint64()
        check(self.L.pow_board_peek(self.ptr, except_slot, tag, ctypes.byref(v)), self.L)
        return None if v.value == 0xFFFFFFFFFFFFFFFF else v.value

    def unlink(self) -> None:
        if self.name:
            check(self.L.pow_board_unlink(self.name.encode()), self.L)

    def close(self) -> None:
        if self.ptr:
            self.L.pow_board_close(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class DeviceBuffer:
    """Device memory owned by a GpuMiner's context (raw pointer for the C ABI)."""

    def __init__(self, miner: "GpuMiner", nbytes: int):
        self.miner, self.nbytes = miner, nbytes
        self.ptr = ctypes.c_void_p()
        check(miner.L.pow_dev_alloc(miner.ctx, nbytes, ctypes.byref(self.ptr)), miner.L)

    def read_u32(self, n: int) -> np.ndarray:
        out = np.zeros(n, dtype=np.uint32)
        if n:
            check(self.miner.L.pow_dev_read(self.miner.ctx, self.ptr, out.ctypes.data_as(ctypes.c_void_p),
                                            4 * n), self.miner.L)
        return out

    def free(self) -> None:
        if self.ptr:
            check(self.miner.L.pow_dev_free(self.miner.ctx, self.ptr), self.miner.L)
            self.ptr = ctypes.c_void_p()


def proof_of_work_round(miner: GpuMiner, last: Block, rank: int, start: int, count: int,
                        difficulty: int = DEFAULT_DIFFICULTY) -> MineResult | None:
    """One round of node.cpp:285-308 on the GPU: template refresh, then the
    nonce -> hash -> test loop over a counter range."""
    return miner.mine(refresh_template(last, rank, difficulty), start, count, difficulty)


def block_hex(b: Block) -> str:
    return field(b, "block_hash").split(b"\0", 1)[0].decode()


__all__ = ["GpuMiner", "DeviceBuffer", "StopBoard", "MineResult", "refresh_template", "proof_of_work_round", "block_hex",
           "nonce_from_counter"]
