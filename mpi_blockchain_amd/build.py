"""Build the in-tree native library ``mpi_blockchain_amd/libpow_gpu.so``.

hipcc cross-compiles for gfx950 only (no GPU needed to build).  The .so is
git-ignored but travels to the GPU box with the gpurun snapshot, so the GPU
tests load exactly this file.

    python -m mpi_blockchain_amd.build [--force]
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libpow_gpu.so")
SOURCES = ["pow_api.cpp", "pow_kernels.hip", "valu_peak.hip"]
HEADERS = ["pow_template.h", "sha256_dev.h"]
INCLUDES = [os.path.join(ROOT, "include", h) for h in ("pow_gpu.h", "pow_tools.h")]
ARCH = "gfx950"


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP toolchain is required to build libpow_gpu.so")


def _inputs() -> list[str]:
    return [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + INCLUDES


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(p) <= t for p in _inputs())


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and up_to_date():
        return LIB
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-fPIC", "-shared", "-std=c++17",
           "-mcode-object-version=5", "-Wall", "-Werror=return-type",
           "-I", os.path.join(ROOT, "include"), "-I", CSRC,
           *[os.path.join(CSRC, s) for s in SOURCES], "-o", LIB + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=ROOT)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
