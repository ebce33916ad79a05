"""Codegen guards for the hot kernel (CPU only: hipcc cross-compiles gfx950).

The mining kernel's speed is set by its instruction stream, so the properties
DESIGN.md relies on are checked on the generated ISA:
  * no scratch, no SGPR/VGPR spills (spilled SGPRs cost a v_readlane each);
  * <= 64 VGPRs -> 8 waves per SIMD;
  * the j-loop body is ~4,850 VALU instructions per trial (SHA-256 of 5
    chunks minus the template-constant and prefix-constant work).
"""
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mpi_blockchain_amd", "csrc")


@pytest.fixture(scope="module")
def isa():
    from mpi_blockchain_amd.build import hipcc

    with tempfile.TemporaryDirectory() as td:
        subprocess.run([hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-mcode-object-version=5",
                        "-I", os.path.join(ROOT, "include"), "-I", CSRC, "-c",
                        os.path.join(CSRC, "pow_kernels.hip"), "-o", os.path.join(td, "k.o"),
                        "-save-temps=obj"], check=True, cwd=td, capture_output=True)
        s = [f for f in os.listdir(td) if f.endswith("gfx950.s")]
        assert s
        return open(os.path.join(td, s[0])).read()


def kernel_body(isa: str, mangled_prefix: str) -> str:
    m = re.search(rf"^({mangled_prefix}\w*):[^\n]*\n(.*?)s_endpgm", isa, flags=re.S | re.M)
    assert m, mangled_prefix
    return m.group(2)


def metadata(isa: str, name_prefix: str) -> dict:
    out = {}
    for blk in isa.split("  - .agpr_count")[1:]:
        nm = re.search(r"\.name:\s+(\S+)", blk)
        if nm and nm.group(1).startswith(name_prefix):
            for key in ("sgpr_spill_count", "vgpr_spill_count", "vgpr_count", "sgpr_count",
                        "private_segment_fixed_size"):
                v = re.search(rf"\.{key}:\s+(\d+)", blk)
                if v:
                    out[key] = int(v.group(1))
            return out
    raise AssertionError(name_prefix)


@pytest.mark.parametrize("variant", ["_Z10pow_searchILi0ELb0E", "_Z10pow_searchILi1ELb0E",
                                     "_Z10pow_searchILi0ELb1E", "_Z10pow_searchILi1ELb1E"])
def test_no_spills_and_occupancy(isa, variant):
    md = metadata(isa, variant)
    assert md["sgpr_spill_count"] == 0
    assert md["vgpr_spill_count"] == 0
    assert md["private_segment_fixed_size"] == 0
    assert md["vgpr_count"] <= 64, md  # 8 waves / SIMD


def test_inner_loop_valu_count(isa):
    body = kernel_body(isa, "_Z10pow_searchILi0ELb0E")
    ops = re.findall(r"^\s+(v_[a-z0-9_]+)", body, flags=re.M)
    n = len(ops)
    # prefix setup + j-loop body (one trial) + epilogue; the trial dominates
    assert 4800 <= n <= 5200, n
    # SGPR spills would show up as hundreds of v_writelane/v_readlane pairs
    assert ops.count("v_readlane_b32") <= 8 and ops.count("v_writelane_b32") == 0
    for needed in ("v_alignbit_b32", "v_bitop3_b32", "v_add3_u32"):
        assert ops.count(needed) > 500, needed
