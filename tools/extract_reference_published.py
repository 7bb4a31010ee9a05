#!/usr/bin/env python3
"""Extract the reference's published per-matrix GFLOP/s (RTX 4090) for the SuiteSparse matrices
this repository rebuilds exactly (bsmr/synth.py SUITESPARSE_REBUILDS).

Runs only in the build container (it reads /root/reference, absent on the GPU box). Output:
tests/golden/reference_published_gflops.json — DATA ONLY: the rows of
scripts/results_suiteSparse_dataset/k<K>/results_<K>.csv (BSMR = best bsmr_gflops over the 35
(alpha, delta) settings, analyze_results.cpp:283-345, and the baselines' columns), with the file
and line each number comes from.
"""
import csv
import json
import os
import sys

SRC = "/root/reference/scripts/results_suiteSparse_dataset"
MATRICES = ["Trefethen_20000", "Trefethen_20000b", "mycielskian14", "mycielskian15", "mycielskian16"]


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(__file__), "..", "tests", "golden", "reference_published_gflops.json")
    rows = []
    for K in (32, 64, 128, 256):
        rel = f"k{K}/results_{K}.csv"
        with open(os.path.join(SRC, rel)) as f:
            lines = f.read().splitlines()
        header = next(csv.reader([lines[0]]))
        for ln, text in enumerate(lines[1:], start=2):
            rec = dict(zip(header, next(csv.reader([text]))))
            name = os.path.basename(rec[header[0]]).rsplit(".", 1)[0]
            if name not in MATRICES:
                continue
            row = {"matrix": name, "K": K, "source": f"scripts/results_suiteSparse_dataset/{rel}:{ln}",
                   "M": int(rec["M"]), "N": int(rec["N"]), "NNZ": int(rec["NNZ"])}
            for col in header[6:]:
                row[col] = float(rec[col])
            rows.append(row)
    rows.sort(key=lambda r: (r["matrix"], r["K"]))
    with open(out_path, "w") as f:
        json.dump({"source": "reference results_<K>.csv (RTX 4090; BSMR = best over alpha x delta)",
                   "hardware": "NVIDIA GeForce RTX 4090", "rows": rows}, f, indent=1)
    print(f"wrote {len(rows)} rows to {out_path}")


if __name__ == "__main__":
    main()
