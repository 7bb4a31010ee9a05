#!/usr/bin/env python3
"""Clustering candidate filter on / off (bsmr_tuning.cluster_filter) on the patterns at or above
its auto threshold: row-reordering time, filter time, permutation hash, cluster count.

    python3 tools/filter_ab.py [--alphas 0.1,0.3,0.5,0.7,0.9]
"""
import argparse
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sddmm-gpu_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--alphas", default="0.3")
    ap.add_argument("--workloads", default="mycielskian16,cop20k_like,reddit_like:0.25")
    args = ap.parse_args()
    from bsmr import Plan, synth

    for w in args.workloads.split(","):
        name, _, scale = w.partition(":")
        if name in synth.SUITESPARSE_REBUILDS:
            M, N, rp, ci = synth.SUITESPARSE_REBUILDS[name]()
        elif scale:
            M, N, rp, ci = getattr(synth, name)(float(scale))
        else:
            M, N, rp, ci = getattr(synth, name)()
        for a in [float(x) for x in args.alphas.split(",")]:
            row = {"workload": w, "M": M, "nnz": len(ci), "alpha": a}
            for f in (1, 0, -1):
                plan = Plan(M, N, rp, ci, alpha=a, delta=0.3, tuning={"cluster_filter": f})
                st = plan.stats()
                rows = plan.array("reorderedRows")
                row["fauto" if f < 0 else f"f{f}"] = {"row_ms": round(st["row_reorder_ms"], 1),
                                "filter_ms": round(st["cluster_filter_ms"], 1),
                                "used": st["cluster_filter_used"], "clusters": st["num_clusters"],
                                "sha": hashlib.sha256(rows.tobytes()).hexdigest()[:16]}
                del plan
            row["same"] = row["f1"]["sha"] == row["f0"]["sha"] == row["fauto"]["sha"]
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
