"""Peer process of tests/test_board_gpu.py::test_board_shared_between_processes.

Opens the named stop board, binds its miner to `slot` for `tag`, prints
"ready", then mines (any-mode, difficulty 64: no solution) a 2^34-counter
range that would take seconds, and prints one JSON line: whether it found
anything, how long the call took and how many trials it ran.  A peer's hit
published on the board must stop it early.

    python tests/board_peer.py <board-name> <slot> <tag>
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mpi_blockchain_amd.block import make_block  # noqa: E402
from mpi_blockchain_amd.miner import GpuMiner, StopBoard  # noqa: E402


def main():
    name, slot, tag = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    # the test library: POW_GRID_PER_CU (set by the caller) leaves half the chip to the finder
    with GpuMiner(0, test_hooks=True) as m, StopBoard(2, name) as board:
        m.warmup()
        m.bind_board(board, slot, tag)
        print("ready", flush=True)
        b = make_block(1, 0, 9, 1700000000, b"")
        t = time.perf_counter()
        r = m.mine(b, 1 << 33, 1 << 34, 64, any_solution=True)
        dt = time.perf_counter() - t
        st = m.stats()
        m.bind_board(None)
        print(json.dumps({"found": r is not None, "secs": dt, "hashes": st["hashes"]}), flush=True)


if __name__ == "__main__":
    main()
