"""Shared helpers for the tests (builds Blocks from golden.json entries)."""
import ctypes

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
