#!/usr/bin/env python3
"""Timeline of the clustering chain (k_cluster, BSMR_DIAG bit 2048): per tile of T clusters its
kernel entry, the moment its first cluster's start was found (it waits for the predecessor
tile's last start), its end, and its window / empty-window / sub-batch counts. Prints launch
boundaries (gaps with no tile alive), the tile lifetime split and how many tiles were alive.

    python3 tools/cluster_trace.py --workload reddit_like --scale 0.25
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sddmm-gpu_amd"))


def pct(x):
    return [round(float(v), 2) for v in np.percentile(x, [0, 10, 50, 90, 100])] if len(x) else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="reddit_like")
    ap.add_argument("--scale", type=float, default=0.25)
    ap.add_argument("--alpha", type=float, default=0.3)
    ap.add_argument("--dump", default="")
    args = ap.parse_args()
    import bsmr
    from bsmr import Plan, synth

    gen = synth.SUITESPARSE_REBUILDS.get(args.workload) or getattr(synth, args.workload)
    M, N, rp, ci = gen(args.scale) if args.workload not in synth.SUITESPARSE_REBUILDS else gen()
    t0 = time.perf_counter()
    tun = {"diag": 2048}
    if os.environ.get("BSMR_CLUSTER_FILTER") in ("0", "1"):
        tun["cluster_filter"] = int(os.environ["BSMR_CLUSTER_FILTER"])
    plan = Plan(M, N, rp, ci, alpha=args.alpha, delta=0.3, tuning=tun)
    wall = time.perf_counter() - t0
    st = plan.stats()
    L = bsmr.lib()
    L.bsmr_debug_trace.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64)]
    n = C.c_uint64()
    L.bsmr_debug_trace(plan.h, None, C.byref(n))
    buf = np.zeros(n.value, np.uint64)
    L.bsmr_debug_trace(plan.h, buf.ctypes.data, C.byref(n))
    t = buf.reshape(-1, 16)
    t = t[t[:, 2] > 0].astype(np.int64)
    if args.dump:
        np.save(args.dump, t)
    us = 0.01
    b, s, e = t[:, 0], t[:, 1], t[:, 2]
    base = b.min()
    # launches: the ticket restarts at 0 in every launch
    starts = np.nonzero(t[:, 7] == 0)[0]
    launches = []
    for k, i0 in enumerate(starts):
        i1 = starts[k + 1] if k + 1 < len(starts) else len(t)
        launches.append({"tiles": int(i1 - i0), "begin_s": round(float((b[i0:i1].min() - base) * us * 1e-6), 3),
                         "end_s": round(float((e[i0:i1].max() - base) * us * 1e-6), 3)})
    gaps = [round(launches[k + 1]["begin_s"] - launches[k]["end_s"], 4) for k in range(len(launches) - 1)]
    # tiles alive over time (sampled at 200 points)
    grid = np.linspace(b.min(), e.max(), 200)
    alive = [int(((b <= g) & (e > g)).sum()) for g in grid]
    out = {"workload": args.workload, "scale": args.scale, "M": M, "nnz": len(ci),
           "plan_wall_s": round(wall, 3), "clusters": st.get("num_clusters"),
           "tiles": int(len(t)), "span_s": round(float((e.max() - base) * us * 1e-6), 3),
           "launches": len(launches), "launch_gap_s_total": round(float(sum(gaps)), 4),
           "wait_for_start_us": pct((s - b) * us), "life_us": pct((e - b) * us),
           "windows": pct(t[:, 3]), "empty_window_frac": round(float(t[:, 4].sum() / max(1, t[:, 3].sum())), 3),
           "subbatches": pct(t[:, 5]), "evals_per_tile": pct(t[:, 6]),
           "exact_evals_total": int(t[:, 11].sum()),
           # candidate filter: rows a tile evaluated (the rest were skipped by their bits), and
           # clusters holding more than their leader row (never skipped)
           "evaluated_rows_total": int(t[:, 14].sum()), "multi_clusters_total": int(t[:, 15].sum()),
           "tiles_with_multi": int((t[:, 15] > 0).sum()),
           "filter_ms": round(float(st.get("cluster_filter_ms", 0.0)), 2),
           # where a tile's life goes (sums over tiles, fraction of summed lifetimes)
           "life_split": {k: round(float(t[:, i].sum() / max(1, (e - b).sum())), 3)
                          for k, i in (("scan_and_spin", 8), ("evaluate", 9), ("leader", 10))},
           "eval_us_per_subbatch": round(float(t[:, 9].sum() * us / max(1, t[:, 5].sum())), 2),
           "lead_us_per_subbatch": round(float(t[:, 10].sum() * us / max(1, t[:, 5].sum())), 2),
           # wave 0's own rows against the whole evaluation phase (the rest: waiting at the
           # barrier for slower waves), and its encoding entries per row / per microsecond
           "wave0_own_frac_of_eval": round(float(t[:, 12].sum() / max(1, t[:, 9].sum())), 3),
           "wave0_entries_per_subbatch": round(float(t[:, 13].sum() / max(1, t[:, 5].sum())), 1),
           "wave0_entries_per_us": round(float(t[:, 13].sum() / max(1e-9, t[:, 12].sum() * us)), 1),
           "alive": {"p10": int(np.percentile(alive, 10)), "p50": int(np.median(alive)),
                     "max": int(max(alive))},
           "first_launches": launches[:3]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
