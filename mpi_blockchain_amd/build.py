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
SOURCES = ["pow_api.cpp", "pow_aql.cpp", "pow_board.cpp", "pow_group.cpp", "pow_kernels.hip", "pow_sort.hip", "valu_peak.hip",
           "pow_test_kernels.hip"]
HEADERS = ["pow_template.h", "sha256_dev.h", "pow_aql.h"]
INCLUDES = [os.path.join(ROOT, "include", h) for h in ("pow_gpu.h", "pow_tools.h")]
ARCH = "gfx950"


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP toolchain is required to build libpow_gpu.so")


def _inputs() -> list[str]:
    return [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + INCLUDES


# Test build: the same kernels and API with -DPOW_TEST_HOOKS, i.e. the test and
# tuning switches read from the environment at pow_init (POW_FORCE_FULL,
# POW_FAULT_INJECT, POW_LAT_MAX, POW_LAT_WPS, POW_GRID_PER_CU) and the RCCL
# library override (POW_TEST_RCCL_LIB, tests/stub_rccl).  The shipped
# libpow_gpu.so has none of them; only tests load this one.
TEST_LIB = os.path.join(PKG, "libpow_gpu_test.so")
OBJ = os.path.join(ROOT, "build", "obj")  # git- and gpurun-ignored: the .so files travel, not the objects
HOOKED = ("pow_api.cpp", "pow_group.cpp")  # the sources that differ between the two builds
# Direct AQL dispatch (round 4's K1'/K2' launch path): linked into the test
# library only, opt-in there with POW_AQL=1.  The shipped library launches
# every kernel through hipLaunchKernel and does not link the HSA runtime.
TEST_ONLY = ("pow_aql.cpp", "pow_test_kernels.hip")  # + the watchdog tests' stall kernel


def _flags() -> list[str]:
    return [f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-mcode-object-version=5", "-Wall",
            "-Werror=return-type", "-I", os.path.join(ROOT, "include"), "-I", CSRC]


def up_to_date(lib: str = LIB) -> bool:
    if not os.path.exists(lib):
        return False
    t = os.path.getmtime(lib)
    return all(os.path.getmtime(p) <= t for p in _inputs())


def _compile(src: str, obj: str, defs: tuple[str, ...], verbose: bool) -> None:
    if os.path.exists(obj) and all(os.path.getmtime(p) <= os.path.getmtime(obj) for p in _inputs()):
        return
    cmd = [hipcc(), *_flags(), *defs, "-c", os.path.join(CSRC, src), "-o", obj + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=ROOT)
    os.replace(obj + ".tmp", obj)


def build(force: bool = False, verbose: bool = False) -> str:
    """libpow_gpu.so (shipped) and libpow_gpu_test.so (tests).  Every source
    is compiled once; pow_api.cpp and pow_group.cpp once more with
    -DPOW_TEST_HOOKS for the test library."""
    if not force and up_to_date(LIB) and up_to_date(TEST_LIB):
        return LIB
    os.makedirs(OBJ, exist_ok=True)
    if force:
        for f in os.listdir(OBJ):
            os.remove(os.path.join(OBJ, f))
    common, plain, hooked = [], [], []
    for s in SOURCES:
        base = os.path.splitext(s)[0]
        if s in TEST_ONLY:
            hooked.append(os.path.join(OBJ, base + ".test.o"))
            _compile(s, hooked[-1], ("-DPOW_TEST_HOOKS",), verbose)
        elif s in HOOKED:
            plain.append(os.path.join(OBJ, base + ".o"))
            hooked.append(os.path.join(OBJ, base + ".test.o"))
            _compile(s, plain[-1], (), verbose)
            _compile(s, hooked[-1], ("-DPOW_TEST_HOOKS",), verbose)
        else:
            common.append(os.path.join(OBJ, base + ".o"))
            _compile(s, common[-1], (), verbose)
    for lib, objs in ((LIB, plain), (TEST_LIB, hooked)):
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *common, *objs, "-o", lib + ".tmp"]
        if lib == TEST_LIB:  # pow_aql.cpp: direct dispatch
            cmd += ["-L", "/opt/rocm/lib", "-lhsa-runtime64", "-Wl,-rpath,/opt/rocm/lib"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True, cwd=ROOT)
        os.replace(lib + ".tmp", lib)
    return LIB


STUB_SRC = os.path.join(ROOT, "tests", "stub_rccl", "stub_rccl.cpp")
STUB_LIB = os.path.join(ROOT, "tests", "stub_rccl", "libstub_rccl.so")


def build_test_stub(force: bool = False, verbose: bool = False) -> str:
    """Test infrastructure: the stand-in RCCL (shared-memory reduction) that the
    TEST library loads through POW_TEST_RCCL_LIB, so pow_group_init runs with
    several ranks on one GPU (tests/test_shard_gpu.py)."""
    if not force and os.path.exists(STUB_LIB) and os.path.getmtime(STUB_SRC) <= os.path.getmtime(STUB_LIB):
        return STUB_LIB
    cmd = ["g++", "-std=c++17", "-O2", "-fPIC", "-shared", "-Wall", "-D__HIP_PLATFORM_AMD__",
           "-I", "/opt/rocm/include", STUB_SRC, "-o", STUB_LIB + ".tmp", "-L", "/opt/rocm/lib", "-lamdhip64",
           "-Wl,-rpath,/opt/rocm/lib"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=ROOT)
    os.replace(STUB_LIB + ".tmp", STUB_LIB)
    return STUB_LIB


MPI_HOME = os.environ.get("POW_MPI_HOME", "/opt/conda")  # the image's MPICH (mpi.h, libmpi.so)
NODE_SRC = os.path.join(CSRC, "node", "pow_node.cpp")
NODE_BIN = os.path.join(PKG, "bin", "pow_node")
# The same node with the protocol tests' race-shaping switches compiled in
# (-DPOW_NODE_TEST_KNOBS: --hold-first, --idle-below, --private-lead, pauses).
# The shipped bin/pow_node behaves only as node.cpp does.
NODE_TEST_BIN = os.path.join(PKG, "bin", "pow_node_test")
NODE_TEST_KNOBS = ("--pause-ms", "--pause-us", "--winner-pause-us", "--hold-first", "--idle-below", "--private-lead",
                   "--lead-barrier", "--recv-delay-rank", "--recv-delay-us")


def mpi_available() -> bool:
    return os.path.exists(os.path.join(MPI_HOME, "include", "mpi.h")) and \
        os.path.exists(os.path.join(MPI_HOME, "lib", "libmpi.so"))


def build_node(force: bool = False, verbose: bool = False, test: bool = False) -> str | None:
    """The protocol node (C++ + MPI) over libpow_gpu.so; skipped without MPI.
    test=True builds bin/pow_node_test (the test knobs compiled in).
    Run it with LD_LIBRARY_PATH=/lib/x86_64-linux-gnu:$MPI_HOME/lib (see
    mpi_blockchain_amd/node.py): MPICH's directory also holds an older
    libstdc++ that must not shadow the system one."""
    if not mpi_available():
        return None
    build(force=False, verbose=verbose)
    out = NODE_TEST_BIN if test else NODE_BIN
    srcs = [NODE_SRC, LIB, os.path.join(ROOT, "include", "pow_gpu.h")]
    if not force and os.path.exists(out) and all(os.path.getmtime(p) <= os.path.getmtime(out) for p in srcs):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = ["g++", "-std=c++17", "-O2", "-pthread", "-Wall", *(["-DPOW_NODE_TEST_KNOBS"] if test else []),
           "-I", os.path.join(ROOT, "include"),
           "-I", os.path.join(MPI_HOME, "include"), NODE_SRC, "-o", out + ".tmp",
           "-L", PKG, "-lpow_gpu", "-Wl,-rpath,$ORIGIN/..",
           os.path.join(MPI_HOME, "lib", "libmpi.so"), f"-Wl,-rpath-link,{os.path.join(MPI_HOME, 'lib')}"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=ROOT)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    print(build_node(force="--force" in sys.argv, verbose=True))
    print(build_node(force="--force" in sys.argv, verbose=True, test=True))
    print(build_test_stub(force="--force" in sys.argv, verbose=True))
