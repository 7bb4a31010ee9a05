#!/usr/bin/env python3
"""HBM traffic (and MFMA activity) per SDDMM launch from a tools/gpu_pmc_config.sh /
tools/gpu_pmc.sh run (separate FETCH_SIZE, WRITE_SIZE, ... passes over tools/prof_sddmm.py),
corrected as MI355X_MICROARCH.md's HBM section prescribes: FETCH_SIZE (KiB) reports half the
bytes of wide reads on gfx950 -> x2; WRITE_SIZE (KiB) as is (exact for 16-B streaming stores; the
4-byte scattered output stores are an uncalibrated width).

Writes the JSON bench.py reads for roofline.traffic, stamped with the sha256 of the kernel and
layout sources it was measured on (bench.py uses it only while they are unchanged).

    python3 tools/pmc_traffic.py gpurun_out/<tag>/C2 profiles/traffic_C2_K128.json
"""
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL_SOURCES = ["sddmm-gpu_amd/csrc/sddmm.hip", "sddmm-gpu_amd/csrc/sddmm_half.hip",
                  "sddmm-gpu_amd/csrc/sddmm_dense.hip", "sddmm-gpu_amd/csrc/plan.hip",
                  "sddmm-gpu_amd/csrc/plan.hpp"]


def kernel_avg_ns(trace_dir):
    """Average duration of the fused launches' kernel from the kernel-trace CSV (the last third
    of the k_sddmm dispatches of prof_sddmm.py: plain, dense-only, residual-only, fused)."""
    import csv
    f = os.path.join(trace_dir, "run_kernel_trace.csv")
    if not os.path.exists(f):
        return None, None
    rows = [r for r in csv.DictReader(open(f)) if "k_sddmm" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    n = (len(rows) - 1) // 3
    full = rows[1 + 2 * n:]
    if not full:
        return None, None
    d = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in full)
    return sum(d) / len(d), full[0]["Kernel_Name"].split("(")[0]


def main(src, dst):
    out = subprocess.check_output([sys.executable, os.path.join(ROOT, "tools", "pmc_table.py"), src])
    t = json.loads(out)
    full = t["full"]
    fetch = 2.0 * full["FETCH_SIZE"] * 1024.0
    write = full["WRITE_SIZE"] * 1024.0
    hashes = {}
    for rel in KERNEL_SOURCES:
        with open(os.path.join(ROOT, rel), "rb") as f:
            hashes[rel] = hashlib.sha256(f.read()).hexdigest()
    res = {"hbm_bytes_per_launch": round(fetch + write),
           "fetch_bytes": round(fetch), "write_bytes": round(write),
           "source": os.path.relpath(src, ROOT),
           "measured_on": os.path.basename(os.path.dirname(os.path.abspath(src))),
           "kernel_sources_sha256": hashes,
           "counters_full_launch": full,
           "note": "median over the fused launches; FETCH_SIZE x2 (gfx950), WRITE_SIZE as reported"}
    avg_ns, kname = kernel_avg_ns(os.path.join(src, "trace"))
    if avg_ns:
        res["kernel"] = kname
        res["kernel_avg_ns_traced"] = round(avg_ns, 1)
        res["hbm_GBps_traced"] = round((fetch + write) / avg_ns, 2)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in full and full.get("GRBM_GUI_ACTIVE"):
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs: wall cycles = /8; 256 CUs x 4 SIMDs
        wall = full["GRBM_GUI_ACTIVE"] / 8.0
        res["mfma"] = {
            "SQ_VALU_MFMA_BUSY_CYCLES": full["SQ_VALU_MFMA_BUSY_CYCLES"],
            "SQ_BUSY_CU_CYCLES": full.get("SQ_BUSY_CU_CYCLES"),
            "GRBM_GUI_ACTIVE": full["GRBM_GUI_ACTIVE"],
            "busy_frac_of_simd_cycles": round(full["SQ_VALU_MFMA_BUSY_CYCLES"] / (wall * 1024.0), 4),
            "busy_frac_of_cu_busy": (round(full["SQ_VALU_MFMA_BUSY_CYCLES"] /
                                           (4.0 * full["SQ_BUSY_CU_CYCLES"]), 4)
                                     if full.get("SQ_BUSY_CU_CYCLES") else None),
            "mops": {k: full[k] for k in full if k.startswith("SQ_INSTS_VALU_MFMA_MOPS")},
            "SQ_INSTS_MFMA": full.get("SQ_INSTS_MFMA"),
        }
    with open(dst, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
