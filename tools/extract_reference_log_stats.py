#!/usr/bin/env python3
"""Extract golden reorder statistics from the reference's own published logs.

Runs only in the build container (it reads /root/reference, which does not exist on the GPU
box). Output: tests/golden/reference_log_stats.json — DATA ONLY (numbers the reference printed),
for the SuiteSparse matrices of those logs that tools/suitesparse_synth.py can rebuild exactly
from their published definitions.

Source: /root/reference/scripts/results_suiteSparse_dataset/BSMR_results/BSMR_k_<K>_a_<a>_d_<d>.log,
one "---New data---" record per matrix, printed by Logger::printLogInformation
(include/Logger.hpp:122-187) in test mode (src/sddmm.cu:62-118).
"""
import json
import os
import re
import sys

LOG_DIR = "/root/reference/scripts/results_suiteSparse_dataset/BSMR_results"
MATRICES = ["Trefethen_20000", "Trefethen_20000b", "mycielskian14", "mycielskian15", "mycielskian16"]
INT_KEYS = [
    "K", "M", "N", "NNZ", "NumRowPanel", "original_numDenseBlock", "bsmr_numClusters",
    "bsmr_numDenseBlock", "bsmr_numDenseThreadBlocks", "bsmr_numSparseThreadBlocks",
    "bsmr_numDenseData", "bsmr_numSparseData",
]
STR_KEYS = ["original_averageDensity", "bsmr_averageDensity", "bsmr_alpha", "bsmr_delta",
            "gridDim_dense", "gridDim_sparse", "bsmr_threadBlockRatio", "bsmr_dataRatio",
            "sparsity", "bsmr_gflops", "bsmr_sddmm"]


def parse_record(text):
    rec = {}
    for key, val in re.findall(r"\[([A-Za-z_]+)\s*: ([^\]]*)\]", text):
        rec[key] = val.strip()
    return rec


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(__file__), "..", "tests", "golden", "reference_log_stats.json")
    records = []
    for fname in sorted(os.listdir(LOG_DIR)):
        m = re.match(r"BSMR_k_(\d+)_a_([\d.]+)_d_([\d.]+)\.log$", fname)
        if not m:
            continue
        with open(os.path.join(LOG_DIR, fname)) as f:
            chunks = f.read().split("---New data---")
        for ch in chunks:
            fm = re.search(r"\[File : [^\]]*/([^/\]]+)\.mtx\]", ch)
            if not fm or fm.group(1) not in MATRICES:
                continue
            rec = parse_record(ch)
            row = {"matrix": fm.group(1), "log": fname}
            for k in INT_KEYS:
                row[k] = int(rec[k])
            for k in STR_KEYS:
                row[k] = rec[k]
            records.append(row)
    records.sort(key=lambda r: (r["matrix"], float(r["bsmr_alpha"]), float(r["bsmr_delta"]), r["K"]))
    os.makedirs(os.path.dirname(os.path.abspath(out_path)), exist_ok=True)
    with open(out_path, "w") as f:
        json.dump({"source": "reference BSMR_results logs (RTX 4090 run, Logger.hpp format)",
                   "records": records}, f, indent=1)
    print(f"wrote {len(records)} records to {out_path}")


if __name__ == "__main__":
    main()
