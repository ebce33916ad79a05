"""Shared helpers for the tests (builds Blocks from golden.json entries)."""
import ctypes
import os
import subprocess
import tempfile

from mpi_blockchain_amd._lib import Block
from mpi_blockchain_amd.block import make_block, set_field


def block_from_template(t: dict) -> Block:
    return make_block(t["index"], t["node_owner_number"], t["difficulty"], t["created_at"],
                      bytes.fromhex(t["previous_block_hash_hex"]))


def block_from_random(e: dict) -> Block:
    b = make_block(e["index"], e["node_owner_number"], e["difficulty"], e["created_at"],
                   bytes.fromhex(e["previous_block_hash_hex"]))
    set_field(b, "nonce", bytes.fromhex(e["nonce_hex"]))
    return b


def with_nonce(b: Block, nonce10: bytes) -> Block:
    c = Block()
    ctypes.pointer(c)[0] = b
    set_field(c, "nonce", nonce10)
    return c


def leading_zero_bits(hexd: str) -> int:
    return 256 - int(hexd, 16).bit_length()


def check_chain(entries, blocks: int, difficulty: int) -> bool:
    """A logged chain (tip first): consecutive indices, linked, every hash
    solving.  Returns True if it is complete (blocks..1, ending at genesis).
    A rank killed by the first finisher's MPI_Abort (node.cpp:330) may leave
    a partial dump; what it did write must still be consistent."""
    idx = [e.index for e in entries]
    assert idx == list(range(idx[0], idx[0] - len(idx), -1)) if idx else True
    for cur, prev in zip(entries, entries[1:]):
        assert cur.prev == prev.hash
    for e in entries:
        assert len(e.hash) == 64 and leading_zero_bits(e.hash) >= difficulty
    return idx == list(range(blocks, 0, -1)) and entries[-1].prev == ""


REF_LOG_CHAIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref",
                             "ref_log_chain")


def reference_dump(entries, rank: int) -> bytes:
    """The bytes the REFERENCE's log_msg + log_chain (node.cpp:40-68, run as
    proof_of_work's termination does, node.cpp:286-289) write for this chain
    (tip first): oracle/_ref/ref_log_chain, built from /root/reference's own
    node.cpp + block.cpp."""
    from mpi_blockchain_amd.node import mpi_env

    tsv = "".join(f"{e.index}\t{e.owner}\t{e.prev}\t{e.hash}\n" for e in entries)
    with tempfile.TemporaryDirectory() as td:
        subprocess.run([REF_LOG_CHAIN, str(rank)], input=tsv.encode(), cwd=td, env=mpi_env(), check=True,
                       capture_output=True, timeout=60)
        return open(os.path.join(td, f"{rank}.out"), "rb").read()
