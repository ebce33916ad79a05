#!/usr/bin/env python3
"""Summarise a profile_round.sh run: per-dispatch averages of the pow_search
kernel from the kernel-trace and PMC CSVs, with the derived quantities DESIGN.md
quotes (VALU instructions per hash, VALUBusy, effective clock, HBM bytes).

    python tools/pmc_summary.py gpurun_out prof_r01 [hashes_per_dispatch] > profiles/r01/pmc_summary.json

gfx950 corrections (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7):
GRBM_GUI_ACTIVE is summed over the 8 XCDs; FETCH_SIZE/WRITE_SIZE are in KiB
and count 64-B memory-side requests — FETCH_SIZE under-reads wide streaming
loads 2x (this kernel has none: its reads are scalar constant loads), and
WRITE_SIZE counts one request per atomic or partial-line store.
"""
import collections
import csv
import glob
import json
import os
import sys

root, tag = sys.argv[1], sys.argv[2]
hashes = float(sys.argv[3]) if len(sys.argv) > 3 else float(1 << 32)
KERNEL = "pow_search<0, false>"
out = {"tag": tag, "kernel": KERNEL, "hashes_per_dispatch": hashes}

kt = glob.glob(os.path.join(root, f"{tag}_kt", "*kernel_trace.csv"))
if kt:
    rows = [r for r in csv.DictReader(open(kt[0])) if KERNEL in r["Kernel_Name"]]
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
    out["dispatches"] = len(rows)
    out["avg_ns"] = sum(durs) / len(durs)
    out["durations_ns"] = durs
    out["vgpr"], out["sgpr"] = rows[0]["VGPR_Count"], rows[0]["SGPR_Count"]
    out["grid"] = rows[0].get("Grid_Size_X") or rows[0].get("Grid_Size")

counters = collections.defaultdict(list)
for f in glob.glob(os.path.join(root, f"{tag}_pmc*", "*counter_collection.csv")):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if KERNEL in r["Kernel_Name"]:
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, c), v in per.items():
        counters[c].append(v)
# Median per dispatch: an occasional dispatch overlaps another process's work
# on the box (one FETCH_SIZE reading of 80 MB among 0.35 MB ones in r02).
avg = {c: sorted(v)[len(v) // 2] for c, v in counters.items()}
out["counters"] = avg
out["per_dispatch"] = {c: v for c, v in counters.items()}
t = out.get("avg_ns")
if "SQ_INSTS_VALU" in avg:
    out["valu_instr_per_hash"] = avg["SQ_INSTS_VALU"] * 64 / hashes
if "GRBM_GUI_ACTIVE" in avg and t:
    per_xcd = avg["GRBM_GUI_ACTIVE"] / 8
    out["clock_ghz"] = per_xcd / t
    if "SQ_ACTIVE_INST_VALU" in avg:
        # counter_defs' VALUBusy prices an instruction at 4 cycles (SIMD-16): > 100 % on
        # gfx950; the raw ratio, and the SIMD-32 scaling (a full-rate instruction = 2 cycles)
        out["sq_active_inst_valu_per_cu_cycle"] = avg["SQ_ACTIVE_INST_VALU"] / 256 / per_xcd
        out["valu_busy_pct_simd32"] = 50 * avg["SQ_ACTIVE_INST_VALU"] / 256 / per_xcd
if "FETCH_SIZE" in avg or "WRITE_SIZE" in avg:
    fb = avg.get("FETCH_SIZE", 0) * 1024
    wb = avg.get("WRITE_SIZE", 0) * 1024
    out["hbm_bytes_per_dispatch"] = {"fetch": fb, "write": wb, "total": fb + wb}
print(json.dumps(out, indent=1))
