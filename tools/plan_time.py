#!/usr/bin/env python3
"""Plan-build timing (row reordering = clustering, column reordering) of a synthetic workload for
several clustering batch sizes; checks that every batch size gives the same permutation.

    python3 tools/plan_time.py --workload reddit_like --scale 0.25 --batches 512,2048
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sddmm-gpu_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="reddit_like")
    ap.add_argument("--scale", type=float, default=None)
    ap.add_argument("--batches", default="512")
    args = ap.parse_args()
    import numpy as np

    from bsmr import Plan, set_default_tuning, synth, tuning_from_env

    set_default_tuning(tuning_from_env())  # BSMR_* knobs (A/B runs)

    gen = getattr(synth, args.workload)
    M, N, rp, ci = gen(args.scale) if args.scale is not None else gen()
    out = {"workload": args.workload, "scale": args.scale, "M": M, "N": N, "nnz": len(ci),
           "runs": {}}
    ref = None
    for b in [int(x) for x in args.batches.split(",")]:
        t0 = time.perf_counter()
        plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, cluster_batch=b)
        wall = time.perf_counter() - t0
        st = plan.stats()
        rows = plan.array("reorderedRows")
        same = None if ref is None else bool(np.array_equal(rows, ref))
        ref = rows if ref is None else ref
        import hashlib
        out["runs"][b] = {"wall_s": round(wall, 3), "row_reorder_ms": round(st["row_reorder_ms"], 2),
                          "rows_sha256": hashlib.sha256(rows.tobytes()).hexdigest()[:16],
                          "lib": os.environ.get("BSMR_LIB_PATH", "in-tree"),
                          "col_reorder_ms": round(st["col_reorder_ms"], 2),
                          "num_clusters": st["num_clusters"],
                          "total_similarity_evals": st["total_similarity_evals"],
                          "exact_similarity_evals": st["exact_similarity_evals"],
                          "cluster_filter_used": st["cluster_filter_used"],
                          "cluster_filter_ms": round(st["cluster_filter_ms"], 2),
                          "same_permutation_as_first": same}
        print(json.dumps({b: out["runs"][b]}), file=sys.stderr, flush=True)
        del plan
    print(json.dumps(out))


if __name__ == "__main__":
    main()
