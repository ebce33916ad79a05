"""MI355X-native proof-of-work miner for the MPI_blockchain protocol.

The reference (CatOfTheCannals/MPI_blockchain) mines in ``proof_of_work``'s
inner loop (node.cpp:292-308): random nonce -> picosha2 SHA-256 of the 270-byte
block serialization -> leading-zero-bit test.  This package puts that loop on
gfx950 behind the C ABI of ``include/pow_gpu.h`` (``libpow_gpu.so``) and keeps
the reference's names on the host side:

* :mod:`mpi_blockchain_amd.block`  — Block model (block.h / block.cpp)
* :mod:`mpi_blockchain_amd.miner`  — GPU miner (proof_of_work's hot loop)
* :mod:`mpi_blockchain_amd.shard`  — nonce space sharded over GPUs, RCCL min
"""
from ._lib import Block, PowError, load  # noqa: F401

__version__ = "0.1.0"
