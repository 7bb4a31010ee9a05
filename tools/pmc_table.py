#!/usr/bin/env python3
"""Summarise a tools/gpu_pmc.sh output directory: per launch kind (grid size / call order of
tools/prof_sddmm.py: dense, residual, full) the median of every counter collected."""
import collections
import csv
import glob
import json
import os
import sys


def main(root):
    out = {}
    for f in sorted(glob.glob(os.path.join(root, "*", "run_counter_collection.csv"))):
        rows = list(csv.DictReader(open(f)))
        per = collections.defaultdict(dict)
        names = {}
        for r in rows:
            d = int(r["Dispatch_Id"])
            per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            names[d] = (r["Kernel_Name"].split("(")[0][-40:], r["Grid_Size"])
        ids = sorted(per)
        # prof_sddmm: 1 plain launch, then iters x dense, iters x residual, iters x full
        n = (len(ids) - 1) // 3
        kinds = {"dense": ids[1:1 + n], "residual": ids[1 + n:1 + 2 * n], "full": ids[1 + 2 * n:]}
        for kind, sel in kinds.items():
            for c in per[sel[0]]:
                vals = sorted(per[i][c] for i in sel)
                out.setdefault(kind, {})[c] = vals[len(vals) // 2]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
