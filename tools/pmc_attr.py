#!/usr/bin/env python3
"""Per-pass summary of a tools/gpu_c4attr.sh directory: the median over the fused launches of each
counter (FETCH_SIZE reported x2 on gfx950, WRITE_SIZE as is; MI355X_MICROARCH.md HBM section), in
GB per launch, and the attribution of the L2-miss (HBM + Infinity Cache) bytes by stream:
staging-only launch (BSMR_DIAG 8), B gathers (full minus the B-in-L2 ablation, DIAG 64), stores
(full minus the no-store ablation, DIAG 128).

    python3 tools/pmc_attr.py gpurun_out/<tag>/c4attr
"""
import collections
import csv
import glob
import json
import os
import sys


def pass_values(d):
    rows = list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
    per = collections.defaultdict(dict)
    for r in rows:
        i = int(r["Dispatch_Id"])
        per[i][r["Counter_Name"]] = per[i].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(per)
    n = (len(ids) - 1) // 3  # tools/prof_sddmm.py: 1 plain, then iters x dense/residual/full
    full = ids[1 + 2 * n:]
    out = {}
    for c in per[full[0]]:
        v = sorted(per[i][c] for i in full)[len(full) // 2]
        if c == "FETCH_SIZE":
            out["fetch_GB"] = round(2.0 * v * 1024 / 1e9, 3)
        elif c == "WRITE_SIZE":
            out["write_GB"] = round(v * 1024 / 1e9, 3)
        else:
            out[c] = v
    return out


def main(root):
    res = {os.path.basename(os.path.dirname(f)): pass_values(os.path.dirname(f))
           for f in sorted(glob.glob(os.path.join(root, "*", "run_counter_collection.csv")))}
    full = res.get("trace_fetch", {}).get("fetch_GB")
    if full is not None:
        attr = {"full_fetch_GB": full}
        if "fetch_stage" in res:
            attr["A_staging_GB (staging-only launch)"] = res["fetch_stage"]["fetch_GB"]
        if "fetch_bl2" in res:
            attr["B_gathers_GB (full - B-in-L2)"] = round(full - res["fetch_bl2"]["fetch_GB"], 3)
        if "fetch_nostore" in res:
            attr["P_store_pass_GB (full - no stores)"] = round(full - res["fetch_nostore"]["fetch_GB"], 3)
        if "tcc" in res:
            h, m = res["tcc"].get("TCC_HIT_sum", 0), res["tcc"].get("TCC_MISS_sum", 0)
            attr["L2_hit_rate"] = round(h / (h + m), 3) if h + m else None
        res["attribution"] = attr
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
