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


def j_loop_body(isa: str, mangled_prefix: str) -> str:
    """The per-trial body: the kernel's largest basic block (one j-step is a
    single ~5k-instruction block of straight-line code)."""
    body = kernel_body(isa, mangled_prefix)
    blocks = re.split(r"^(?:\.LBB\w+:|; %bb\.\d+:).*$", body, flags=re.M)
    return max(blocks, key=lambda b: len(re.findall(r"^\s+v_", b, flags=re.M)))


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
    # SGPRs are capped at 80 (8 workgroups/CU); the few spills this causes sit
    # at chunk-dequeue level and in the rare hit path, never in the j-loop
    # (test_j_loop_clean).
    # (mine modes also keep the early-exit / cancellation poll state: <= 24)
    assert md["sgpr_spill_count"] <= (16 if "ILi0E" in variant else 24)
    assert md["vgpr_spill_count"] == 0
    assert md["private_segment_fixed_size"] == 0
    assert md["vgpr_count"] <= 64, md  # 8 waves / SIMD


@pytest.mark.parametrize("variant", ["_Z10pow_searchILi0ELb0E", "_Z10pow_searchILi1ELb0E"])
def test_j_loop_clean(isa, variant):
    body = j_loop_body(isa, variant)
    ops = re.findall(r"^\s+([sv]_[a-z0-9_]+|ds_\w+|flat_\w+|global_\w+|scratch_\w+|buffer_\w+)", body, flags=re.M)
    valu = [o for o in ops if o.startswith("v_")]
    # one trial: chunk-0 rounds 4..63 + schedule, chunks 1-4, test = 4,831 VALU
    # (PMC: 4,837 per hash with the per-chunk work, profiles/r02/final)
    assert 4800 <= len(valu) <= 4860, len(valu)
    assert "v_readlane_b32" not in ops and "v_writelane_b32" not in ops
    assert not [o for o in ops if o.startswith(("flat_", "global_", "scratch_", "buffer_"))], \
        "the j-loop must take its constants through scalar and LDS loads only"
    # chunk 0's uniform words (K[16..63], K+W[4..15], the j terms) arrive by
    # scalar loads; chunks 1-4's 4 x 64 K+W words by LDS broadcast reads into
    # VGPRs (no SGPR operand in their K+W adds)
    words = sum({"s_load_dwordx16": 16, "s_load_dwordx8": 8, "s_load_dwordx4": 4, "s_load_dwordx2": 2,
                 "s_load_dword": 1}.get(o, 0) for o in ops)
    assert words >= 48 + 12, words
    assert ops.count("ds_read_b128") == 64, ops.count("ds_read_b128")
    sgpr_adds = len(re.findall(r"^\s+v_add_u32_e32 [^\n]*\bs\d+", body, flags=re.M))
    assert sgpr_adds <= 16, sgpr_adds


def test_k2_fits_beside_k1(isa):
    """K2 (block validation) must fit in the one workgroup slot K1 leaves free
    (pow_api.cpp: grid = 8 x CUs - 1): a SIMD then has 512 - 7 x 64 = 64 VGPRs
    for it.  No scratch either."""
    md = metadata(isa, "_Z15pow_hash_kernel")
    assert md["vgpr_count"] <= 64, md
    assert md["vgpr_spill_count"] == 0 and md["private_segment_fixed_size"] == 0, md


def test_k2_one_block_fits_beside_k1(isa):
    """K2' (pow_hash_block's one-block path) runs in the same free workgroup
    slot as K2: <= 64 VGPRs, no scratch (its by-value message is read through
    the kernarg pointer, not copied), LDS only for the five K+W schedules."""
    md = metadata(isa, "_Z12pow_hash_one")
    assert md["vgpr_count"] <= 64, md
    assert md["vgpr_spill_count"] == 0 and md["private_segment_fixed_size"] == 0, md


@pytest.mark.parametrize("variant", ["_Z14pow_search_latILb0ELb0E", "_Z14pow_search_latILb0ELb1E"])
def test_latency_kernel_no_private_copy(isa, variant):
    """The latency kernel reads its by-value constants through the kernarg
    pointer; taking the parameter's address would copy 2.3 KB to scratch."""
    md = metadata(isa, variant)
    assert md["private_segment_fixed_size"] == 0 and md["vgpr_spill_count"] == 0, md
    # it runs at <= 4 waves per SIMD (pow_api.cpp run_search_lat): <= 128 VGPRs
    assert md["vgpr_count"] <= 128, md
    # chunks 1-4's K+W come from the LDS copy inside the loop, as in K1 (hoisted
    # out of it, the 256 words would take 256 VGPRs)
    body = j_loop_body(isa, variant)
    assert len(re.findall(r"^\s+ds_read_b128", body, flags=re.M)) == 64
    # one trial per lane, nothing hoisted across j: 5,083 VALU (K1: 4,831)
    assert 5000 <= len(re.findall(r"^\s+v_", body, flags=re.M)) <= 5120


def test_trial_issue_mix_matches_bench(isa):
    """bench.py's mix-adjusted ceiling prices K1's trial by its issue classes
    (TRIAL_HALF_RATE / TRIAL_FULL_RATE); they must be the ISA's: half rate =
    v_alignbit_b32, v_add3_u32 and any other op with an SGPR operand."""
    import sys

    sys.path.insert(0, ROOT)
    import bench

    body = j_loop_body(isa, "_Z10pow_searchILi0ELb0E")
    lines = [ln.strip() for ln in body.splitlines() if re.match(r"\s+v_", ln)]
    half = [ln for ln in lines if ln.split()[0] in ("v_alignbit_b32", "v_add3_u32")
            or re.search(r"\bs\d+\b|\bs\[", ln)]
    assert (len(half), len(lines) - len(half)) == (bench.TRIAL_HALF_RATE, bench.TRIAL_FULL_RATE)


def test_valu_microbench_streams():
    """pow_valu_rate's three loops issue exactly the instruction kinds they are
    named for, in the proportions the rate computation assumes, with VGPR
    operands only and 8-byte encodings (no 4-byte VOP2 op: among VOP3 ops it
    issues at half rate, profiles/r03/probe/): MIX is K1's SHA round
    (6 alignbit : 4 bitop3 : 2 add3 : 2 add), FULL bitop3 + add, HALF
    alignbit + add3."""
    import collections

    from mpi_blockchain_amd.build import hipcc

    with tempfile.TemporaryDirectory() as td:
        subprocess.run([hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-mcode-object-version=5",
                        "-I", os.path.join(ROOT, "include"), "-I", CSRC, "-c",
                        os.path.join(CSRC, "valu_peak.hip"), "-o", os.path.join(td, "v.o"),
                        "-save-temps=obj"], check=True, cwd=td, capture_output=True)
        s = open(os.path.join(td, [f for f in os.listdir(td) if f.endswith("gfx950.s")][0])).read()
    want = {"ILi0E": {"v_alignbit_b32": 6, "v_bitop3_b32": 4, "v_add3_u32": 2, "v_add_u32_e64": 2},
            "ILi1E": {"v_bitop3_b32": 1, "v_add_u32_e64": 1},
            "ILi2E": {"v_alignbit_b32": 1, "v_add3_u32": 1}}
    for k, kinds in want.items():
        body = j_loop_body(s, "_Z16valu_rate_kernel" + k)
        ops = [ln.strip() for ln in body.splitlines() if re.match(r"\s+v_", ln)]
        c = collections.Counter(o.split()[0] for o in ops)
        assert set(c) == set(kinds), (k, c)
        unit = c[next(iter(kinds))] // kinds[next(iter(kinds))]
        assert unit > 0 and all(c[op] == n * unit for op, n in kinds.items()), (k, c)
        assert not [o for o in ops if re.search(r"\bs\d+\b|\bs\[", o)], k


@pytest.mark.parametrize("variant", ["_Z10pow_searchILi0ELb0E", "_Z10pow_searchILi1ELb0E", "_Z10pow_searchILi2ELb0E",
                                     "_Z10pow_searchILi0ELb1E"])
def test_trial_block_phase_pinned(isa, variant):
    """The trial block starts on an 8-byte boundary (.p2align 3 at its head):
    the same block 4 bytes off that phase ran ~1.1% slower
    (profiles/r03/ab/ab3_code_placement.log), and the phase would otherwise
    follow whatever code precedes the loop.  The rounds then run as asm
    groups of 4, each pinned by its own .p2align 3: chunk 0's rounds 4-63 (15
    groups) and chunks 1-4 (64 groups), 1 + 15 + 64 in all."""
    body = j_loop_body(isa, variant)
    assert body.count(".p2align 3") == 80, body.count(".p2align 3")
    head = body.split(".p2align 3")[0]
    # the first directive sits at the head of the block: only the per-j scalar set-up precedes it
    assert len(re.findall(r"^\s+v_", head, flags=re.M)) <= 8, head[-2000:]


@pytest.fixture(scope="module")
def k1_code():
    """(address, mnemonic, bytes) of K1's sweep kernel in the assembled gfx950
    code object (the .s has no addresses)."""
    from mpi_blockchain_amd.build import hipcc

    with tempfile.TemporaryDirectory() as td:
        co = os.path.join(td, "k.co")
        subprocess.run([hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-mcode-object-version=5",
                        "-I", os.path.join(ROOT, "include"), "-I", CSRC, "--cuda-device-only",
                        "--no-gpu-bundle-output", "-c", os.path.join(CSRC, "pow_kernels.hip"), "-o", co],
                       check=True, cwd=td, capture_output=True)
        dis = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", co], check=True, capture_output=True,
                             text=True).stdout
    lines = dis.splitlines()
    fn = "_Z10pow_searchILi0ELb0EEvPK9PowConsts9PowLaunchPjP9PowResult"
    i = [k for k, ln in enumerate(lines) if ln.endswith("<" + fn + ">:")][0]
    end = next((k for k in range(i + 1, len(lines)) if re.match(r"^[0-9a-f]{16} <_Z", lines[k])), len(lines))
    out = []
    for ln in lines[i:end]:
        m = re.match(r"^\s+(\S+).*//\s*([0-9A-Fa-f]+):\s*([0-9A-Fa-f ]+)$", ln)
        if m:
            out.append((int(m.group(2), 16), m.group(1), 4 * len(m.group(3).split())))
    return out


def test_chunk_rounds_keep_one_phase(k1_code):
    """Chunks 1-4 (3,600 of a trial's ~4,840 VALU instructions): every
    instruction of the 64 asm groups is 8 bytes long and starts 4 bytes past
    an 8-byte boundary.  That phase issued ~5% faster in the probes
    (tools/place_probe*.hip) and the groups 4.1% faster in K1
    (profiles/r03/ab/ab8_asm_groups_chunks14.log) than hipcc's mixed
    4/8-byte encodings, whose phase flipped at every 4-byte instruction."""
    ds_all = [k for k, (a, op, sz) in enumerate(k1_code) if op == "ds_read_b128"]
    # the trial's 64 reads: the longest run of ds_read_b128 one group (~60 instructions) apart
    runs, cur = [], [ds_all[0]]
    for k in ds_all[1:]:
        if k - cur[-1] < 200:
            cur.append(k)
        else:
            runs.append(cur)
            cur = [k]
    runs.append(cur)
    # (the sweep's flush of staged solutions right after the trial reads LDS 16 B per lane too)
    ds = max(runs, key=len)[:64]
    assert len(ds) == 64, [len(r) for r in runs]
    chunk = [x for x in k1_code[ds[0]:ds[-1] + 60] if x[1].startswith("v_")]
    eight = [x for x in chunk if x[2] == 8]
    off = [x for x in eight if x[0] % 8 != 4]
    assert len(eight) >= 3584 and len(off) <= 32, (len(eight), len(off))


@pytest.mark.parametrize("variant", ["_Z10pow_searchILi0ELb0E", "_Z10pow_searchILi1ELb0E"])
def test_trial_is_asm_groups(isa, variant):
    """Every SHA-256 round and schedule word of the trial is in the asm groups
    (8-byte encodings at the pinned phase); outside them the compiler emits
    only the per-j set-up, the IV feed-forward of chunk 0 and the test:
    <= 16 VALU instructions (round 2: ~135, with 4-byte encodings; a 4-byte
    VOP2 op among 8-byte VOP3 ops issues at half rate, profiles/r03/probe/)."""
    body = j_loop_body(isa, variant)
    outside = re.sub(r";;#ASMSTART.*?;;#ASMEND", "", body, flags=re.S)
    assert len(re.findall(r"^\s+v_", outside, flags=re.M)) <= 16


@pytest.mark.parametrize("variant", ["_Z14pow_search_latILb0ELb0ELb1E", "_Z14pow_search_latILb0ELb1ELb1E"])
def test_latency_kernel_asm_variant(isa, variant):
    """K1' at 4 waves per SIMD runs chunks 1-4 as K1's asm groups: the
    variant fits 4 waves per SIMD (<= 128 VGPRs) without scratch, and keeps
    the 64 LDS reads inside the loop."""
    md = metadata(isa, variant)
    assert md["vgpr_count"] <= 128 and md["private_segment_fixed_size"] == 0 and md["vgpr_spill_count"] == 0, md
    body = j_loop_body(isa, variant)
    assert len(re.findall(r"^\s+ds_read_b128", body, flags=re.M)) == 64
    assert body.count(".p2align 3") == 64


def test_k2_one_block_is_the_rounds_only(isa):
    """K2' (round 4): the host expands the message schedules (K folded in), so
    the kernel is the 320 compression rounds of one block, 14 VALU each in asm
    groups (the compiler's form takes 16), plus the feed-forward: ~4,565 VALU
    (round 3: ~5,100 with the schedules on the device).  Its 80 K+W reads
    (ds_read_b128) are each issued one group ahead of their use."""
    body = kernel_body(isa, "_Z12pow_hash_one")
    assert 4480 <= len(re.findall(r"^\s+v_", body, flags=re.M)) <= 4620
    assert len(re.findall(r"^\s+ds_read_b128", body, flags=re.M)) == 80
    assert len(re.findall(r"^\s+v_add3_u32", body, flags=re.M)) == 2 * 320


AQL_KERNELS = ["_Z12pow_hash_one6PowMsgP10PowHashOutj"] + [
    f"_Z14pow_search_latILb{f}ELb{a}ELb{g}EEv12PowConstsLat12PowLaunchLatP9PowResultS3_"
    for g in (0, 1) for a in (0, 1) for f in (0, 1)]


def test_direct_dispatch_kernels_take_explicit_args_only(isa):
    """pow_aql.cpp writes exactly the kernels' explicit arguments into a packet's
    kernarg slot (PowMsg + pointer + seq = 1,292 B; PowConstsLat + PowLaunchLat
    + 2 pointers = 1,568 B) and nothing the HIP runtime would add: no kernel it
    dispatches may read hidden arguments (gridDim, blockDim, printf buffer...)."""
    for name in AQL_KERNELS:
        blk = next(b for b in isa.split("  - .agpr_count")[1:] if re.search(rf"\.name:\s+{name}\s", b))
        size = int(re.search(r"\.kernarg_segment_size:\s+(\d+)", blk).group(1))
        assert size == (1292 if "hash_one" in name else 1568), (name, size)
        assert "hidden_" not in blk, name


def test_library_embeds_its_code_object():
    """pow_aql.cpp (test library only, POW_AQL=1) loads the kernels from the
    gfx950 code object in the offload bundle of its own .so file: the test
    library holds one that names every kernel it dispatches (the same scan as
    own_code_object)."""
    from mpi_blockchain_amd import _lib

    for path in (_lib.TEST_LIB_PATH,):
        data = open(path, "rb").read()
        found = None
        i = data.find(b"__CLANG_OFFLOAD_BUNDLE__")
        while i >= 0 and found is None:
            n = int.from_bytes(data[i + 24:i + 32], "little")
            off = i + 32
            for _ in range(min(n, 16)):
                o, sz, tl = (int.from_bytes(data[off + 8 * k:off + 8 * k + 8], "little") for k in range(3))
                triple = data[off + 24:off + 24 + tl]
                off += 24 + tl
                co = data[i + o:i + o + sz]
                if triple == b"hipv4-amdgcn-amd-amdhsa--gfx950" and b"_Z12pow_hash_one" in co:
                    found = co
            i = data.find(b"__CLANG_OFFLOAD_BUNDLE__", i + 1)
        assert found is not None and found[:4] == b"\x7fELF", path
        for name in AQL_KERNELS:
            assert (name + ".kd").encode() in found, (path, name)


def _vgprs(operands: str) -> set:
    regs = set()
    for a, b in re.findall(r"\bv\[(\d+):(\d+)\]", operands):
        regs.update(range(int(a), int(b) + 1))
    for a in re.findall(r"\bv(\d+)\b", operands):
        regs.add(int(a))
    return regs


def test_asm_lds_reads_waited_before_use(isa):
    """const_chunks_lds_pipelined (K2', the consensus-critical pow_hash_block)
    issues each K+W read as an asm ds_read_b128 one group ahead and waits for
    it with a separate asm s_waitcnt lgkmcnt(0).  The compiler's waitcnt
    insertion does not track loads issued from inline asm, so a copy, spill or
    reuse of the destination VGPRs placed between the two statements would
    read (or be overwritten by) a load still in flight.  On the generated
    gfx950 code: between every asm ds_read_b128 and the next lgkmcnt(0) wait,
    no instruction names any of its four destination VGPRs."""
    body = kernel_body(isa, "_Z12pow_hash_one")
    pending, reads, checked = set(), 0, 0
    in_asm = False
    for ln in body.splitlines():
        s = ln.strip()
        if s.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        op, _, rest = s.partition(" ")
        rest = rest.split(";")[0]
        if op == "s_waitcnt" and "lgkmcnt(0)" in rest:
            pending = set()
            continue
        regs = _vgprs(rest)
        if op == "ds_read_b128" and in_asm:
            dst = _vgprs(rest.split(",")[0])
            assert len(dst) == 4, s
            assert not (pending & regs), f"a second read reuses in-flight registers: {s}"
            pending |= dst
            reads += 1
            continue
        if pending:
            checked += 1
            assert not (pending & regs), f"{s} touches VGPRs of an asm LDS read still in flight"
    assert reads == 80 and checked > 4000, (reads, checked)  # 5 chunks x 16 groups of 4 K+W words


def test_k1_instruction_budget_guard(isa):
    """K1 stops here (the half-rate instruction mix bounds it at
    0.58 of the SIMD-32 peak, 0.96 of the mix-adjusted ceiling; no GPU time is
    spent on it any more).  This guard catches a regression on the CPU: the
    trial stays at 4,839 VALU instructions (+-1%), of which at most 2,774
    issue at half rate (v_alignbit_b32, v_add3_u32, or an SGPR operand)."""
    for variant in ("_Z10pow_searchILi0ELb0E", "_Z10pow_searchILi1ELb0E", "_Z10pow_searchILi2ELb0E"):
        body = j_loop_body(isa, variant)
        lines = [ln.strip() for ln in body.splitlines() if re.match(r"\s+v_", ln)]
        half = [ln for ln in lines if ln.split()[0] in ("v_alignbit_b32", "v_add3_u32")
                or re.search(r"\bs\d+\b|\bs\[", ln)]
        assert abs(len(lines) - 4839) <= 48, (variant, len(lines))
        assert len(half) <= 2774, (variant, len(half))


# ---- queue pressure guard: no HIP null-stream use in the library's sources ----
# A process that touches HIP's null stream holds one hardware queue more for
# the rest of its life; with 6-8 ranks per GPU that tipped the GPU past its
# compute queue slots and a launch waited 10 s for a queue (round 5,
# DESIGN.md §7 "Queue pressure").  Every copy, fill, event and launch must name
# a stream of its own.
NULL_STREAM_FREE = ("hipMemcpy", "hipMemset", "hipMemsetD8", "hipMemsetD16", "hipMemsetD32", "hipMemcpy2D",
                    "hipMemcpy3D", "hipMemcpyToSymbol", "hipMemcpyFromSymbol", "hipMemcpyHtoD", "hipMemcpyDtoH",
                    "hipMemcpyDtoD", "hipMemcpyPeer", "hipDeviceSynchronize")
# call -> (index of its stream argument, number of arguments with the stream given)
STREAM_ARG = {"hipMemcpyAsync": (4, 5), "hipMemsetAsync": (3, 4), "hipMemsetD32Async": (3, 4),
              "hipMemcpyToSymbolAsync": (5, 6), "hipMemcpyFromSymbolAsync": (5, 6), "hipMemcpy2DAsync": (7, 8),
              "hipMemcpyPeerAsync": (5, 6), "hipEventRecord": (1, 2), "hipLaunchKernelGGL": (4, None),
              "hipExtLaunchKernelGGL": (4, None), "hipLaunchKernel": (5, 6), "hipLaunchCooperativeKernel": (5, 6),
              "hipModuleLaunchKernel": (9, None), "hipStreamSynchronize": (0, 1), "hipStreamQuery": (0, 1),
              "hipStreamWaitEvent": (0, 3), "hipGraphLaunch": (1, 2)}
NULL_STREAMS = {"0", "0u", "nullptr", "NULL", "hipStreamDefault", "hipStreamLegacy", "hipStreamPerThread",
                "(hipStream_t)0", "hipStream_t(0)", "hipStream_t{}", "(hipStream_t) 0"}
SHIPPED_SOURCES = [os.path.join(CSRC, f) for f in ("pow_api.cpp", "pow_aql.cpp", "pow_board.cpp", "pow_group.cpp",
                                                    "pow_kernels.hip", "pow_sort.hip", "valu_peak.hip",
                                                    "pow_test_kernels.hip", "pow_template.h", "sha256_dev.h",
                                                    "pow_aql.h", os.path.join("node", "pow_node.cpp"))] + \
    [os.path.join(ROOT, "tests", "stub_rccl", "stub_rccl.cpp")]


def _strip_comments_and_strings(text: str) -> str:
    """C/C++ source with comments and string/char literals blanked (newlines kept)."""
    out, i, n = [], 0, len(text)
    while i < n:
        c = text[i]
        if text.startswith("//", i):
            j = text.find("\n", i)
            i = n if j < 0 else j
        elif text.startswith("/*", i):
            j = text.find("*/", i + 2)
            j = n if j < 0 else j + 2
            out.append("".join(ch if ch == "\n" else " " for ch in text[i:j]))
            i = j
        elif c in "\"'":
            j = i + 1
            while j < n and text[j] != c:
                j += 2 if text[j] == "\\" else 1
            out.append(c + " " * (min(j, n) - i - 1) + c)
            i = j + 1
        else:
            out.append(c)
            i += 1
    return "".join(out)


def _call_args(text: str, open_paren: int) -> list[str] | None:
    """Top-level arguments of the call whose '(' is at `open_paren`."""
    depth, args, cur = 0, [], []
    for ch in text[open_paren:]:
        if ch in "([{":
            depth += 1
            if depth == 1:
                continue
        elif ch in ")]}":
            depth -= 1
            if depth == 0:
                args.append("".join(cur).strip())
                return [a for a in args if a] if args != [""] else []
        elif ch == "," and depth == 1:
            args.append("".join(cur).strip())
            cur = []
            continue
        cur.append(ch)
    return None


def null_stream_calls(text: str) -> list[tuple[int, str]]:
    """(line, call) of every HIP call in `text` that runs on the null stream:
    a null-stream-only API, a stream argument left out or given as 0/nullptr,
    or a <<<...>>> launch without a stream."""
    src = _strip_comments_and_strings(text)
    bad = []
    line = lambda pos: src.count("\n", 0, pos) + 1  # noqa: E731
    for m in re.finditer(r"\b(hip\w+)\s*\(", src):
        name = m.group(1)
        if name in NULL_STREAM_FREE:
            bad.append((line(m.start()), name))
        elif name in STREAM_ARG:
            args = _call_args(src, m.end() - 1)
            if args is None:
                continue
            idx, full = STREAM_ARG[name]
            if len(args) <= idx or (full is not None and len(args) < full):
                bad.append((line(m.start()), f"{name} without a stream"))
            elif re.sub(r"\s+", " ", args[idx]) in NULL_STREAMS:
                bad.append((line(m.start()), f"{name} on stream {args[idx]}"))
    for m in re.finditer(r"<<<(.*?)>>>", src, re.S):
        cfg = _call_args("(" + m.group(1) + ")", 0) or []
        if len(cfg) < 4 or re.sub(r"\s+", " ", cfg[3]) in NULL_STREAMS:
            bad.append((line(m.start()), "<<<>>> launch on the null stream"))
    return bad


def test_no_null_stream_in_library_sources():
    found = {}
    for p in SHIPPED_SOURCES:
        hits = null_stream_calls(open(p).read())
        if hits:
            found[os.path.relpath(p, ROOT)] = hits
    assert not found, found


def test_null_stream_check_catches_seeded_calls():
    """The guard fails on each form a null-stream call can take (seeded into
    the real valu_peak.hip), and passes the stream-explicit forms."""
    base = open(os.path.join(CSRC, "valu_peak.hip")).read()
    assert null_stream_calls(base) == []
    seeds = ["hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);",
             "hipMemset(d, 0, 8);",
             "hipDeviceSynchronize();",
             "hipMemcpyAsync(h, d, 8, hipMemcpyDeviceToHost);",
             "hipMemcpyAsync(h, d, 8, hipMemcpyDeviceToHost, 0);",
             "hipMemsetAsync(d, 0, 8);",
             "hipEventRecord(e0);",
             "hipEventRecord(e0, nullptr);",
             "hipLaunchKernelGGL((k<1, 2>), dim3(1), dim3(64), 0, 0, a, b);",
             "k<<<dim3(1), dim3(64)>>>(a);",
             "k<<<1, 64, 0, 0>>>(a);",
             "hipStreamSynchronize(0);"]
    for seed in seeds:
        hits = null_stream_calls(base + "\nvoid seeded() {\n  " + seed + "\n}\n")
        assert len(hits) == 1, (seed, hits)
    for ok in ["hipMemcpyAsync(h, d, 8, hipMemcpyDeviceToHost, st);", "hipEventRecord(e0, ctx->stream);",
               "hipLaunchKernelGGL((k<1, 2>), dim3(1), dim3(64), 0, stream, a, b);", "k<<<1, 64, 0, st>>>(a);",
               "// hipMemcpy(h, d, 8, hipMemcpyDeviceToHost); in a comment", 'puts("hipMemset(d, 0, 8)");']:
        assert null_stream_calls("void f() {\n  " + ok + "\n}\n") == [], ok
