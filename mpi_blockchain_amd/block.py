"""The reference's Block model (block.h / block.cpp) over the native library.

Same names and meaning as the reference's free functions (block.h:27-34), so a
caller of the reference finds them here:

=========================  ====================================================
reference                  here
=========================  ====================================================
``struct Block``           :class:`Block` (ctypes, byte-identical, 552 B)
``block_to_str``           :func:`block_to_str` (270 bytes, traps T1/T2)
``block_to_hash``          :meth:`mpi_blockchain_amd.miner.GpuMiner.block_to_hash`
                           (GPU; needs a device context)
``solves_problem``         :func:`solves_problem` (run-time difficulty)
``gen_random_nonce``       :func:`gen_random_nonce` (same alphabet, seeded RNG) and
                           :func:`nonce_from_counter` (the GPU path's counter map)
=========================  ====================================================
"""
from __future__ import annotations

import ctypes
import random

from ._lib import HASH_SIZE, MSG_BYTES, NONCE_SIZE, Block, check, load

# block.h:4-9, node.h:7-10
DEFAULT_DIFFICULTY = 9
BLOCKS_TO_MINE = 10
VALIDATION_MINUTES = 1
VALIDATION_BLOCKS = 5
TAG_NEW_BLOCK = 10
TAG_CHAIN_HASH = 21
TAG_CHAIN_RESPONSE = 22
MAX_BLOCKS = 200

ALPHABET = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789"

__all__ = ["Block", "make_block", "block_to_str", "solves_problem", "nonce_from_counter",
           "gen_random_nonce", "field", "set_field", "DEFAULT_DIFFICULTY", "BLOCKS_TO_MINE",
           "VALIDATION_MINUTES", "VALIDATION_BLOCKS", "HASH_SIZE", "NONCE_SIZE", "MSG_BYTES"]


def field(b: Block, name: str) -> bytes:
    """Raw bytes of a char[] field (ctypes' attribute access stops at NUL)."""
    f = getattr(Block, name)
    return ctypes.string_at(ctypes.addressof(b) + f.offset, f.size)


def set_field(b: Block, name: str, data: bytes) -> None:
    f = getattr(Block, name)
    data = bytes(data)[: f.size].ljust(f.size, b"\0")
    ctypes.memmove(ctypes.addressof(b) + f.offset, data, f.size)


def make_block(index: int = 0, owner: int = 0, difficulty: int = DEFAULT_DIFFICULTY, created_at: int = 0,
               prev: bytes = b"", nonce: bytes = b"", block_hash: bytes = b"") -> Block:
    b = Block()
    b.index = index & 0xFFFFFFFF
    b.node_owner_number = owner & 0xFFFFFFFF
    b.difficulty = difficulty & 0xFFFFFFFF
    b.created_at = created_at & 0xFFFFFFFFFFFFFFFF
    set_field(b, "previous_block_hash", prev)
    set_field(b, "nonce", nonce)
    set_field(b, "block_hash", block_hash)
    return b


def block_to_str(b: Block) -> bytes:
    """block.cpp:79-88: the exact 270-byte message the reference hashes."""
    out = ctypes.create_string_buffer(MSG_BYTES)
    check(load().pow_block_to_bytes(ctypes.byref(b), out))
    return out.raw


def solves_problem(hex_digest: str | bytes, difficulty: int = DEFAULT_DIFFICULTY) -> bool:
    """block.cpp:91-96 with the difficulty (leading zero BITS) as an argument."""
    if isinstance(hex_digest, str):
        hex_digest = hex_digest.encode()
    return bool(load().pow_solves_problem(hex_digest, difficulty))


def nonce_from_counter(ctr: int) -> bytes:
    """Counter -> nonce[10]: 9 base-62 chars (MSB first, alphabet of
    block.cpp:61-72) + NUL."""
    out = ctypes.create_string_buffer(NONCE_SIZE)
    check(load().pow_nonce_from_counter(ctr, out))
    return out.raw


def gen_random_nonce(rng: random.Random | None = None) -> bytes:
    """block.cpp:61-72 with a Python RNG in place of glibc rand()."""
    rng = rng or random
    return "".join(ALPHABET[rng.randrange(62)] for _ in range(NONCE_SIZE - 1)).encode() + b"\0"
