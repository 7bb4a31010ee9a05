#!/usr/bin/env python3
"""Back-to-back runs of one kernel in a rocprofv3 kernel trace: dispatches whose idle gap (start
minus the previous dispatch's end) stays under --gap-us form a run (a replayed HIP graph of K steps is one run of K; Python
stream launches are ~10 us apart and break up). For every run of at least --min launches: mean /
median duration, mean start-to-start interval and span / launches (what HIP events around the run
measure, minus the graph-launch latency before its first kernel).

    python3 tools/rocprof_runs.py <run_kernel_trace.csv> [--kernel k_sddmm_rb] [--min 20]
"""
import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="k_sddmm_rb")
    ap.add_argument("--min", type=int, default=20)
    ap.add_argument("--gap-us", type=float, default=2.0)
    args = ap.parse_args()
    rows = [r for r in csv.DictReader(open(args.trace)) if args.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    st = [int(r["Start_Timestamp"]) for r in rows]
    en = [int(r["End_Timestamp"]) for r in rows]
    runs, a = [], 0
    for i in range(1, len(rows) + 1):
        if i == len(rows) or st[i] - en[i - 1] > args.gap_us * 1e3:
            if i - a >= args.min:
                runs.append((a, i))
            a = i
    out = {"kernel": args.kernel, "dispatches": len(rows),
           "all_mean_duration_us": round(statistics.mean(e - s for s, e in zip(st, en)) / 1e3, 3) if rows else None,
           "runs": []}
    for a, b in runs:
        dur = [en[i] - st[i] for i in range(a, b)]
        gaps = [st[i] - st[i - 1] for i in range(a + 1, b)]
        out["runs"].append({"first_dispatch": a, "n": b - a,
                            "mean_duration_us": round(statistics.mean(dur) / 1e3, 3),
                            "median_duration_us": round(statistics.median(dur) / 1e3, 3),
                            "mean_start_to_start_us": round(statistics.mean(gaps) / 1e3, 3),
                            "span_per_launch_us": round((en[b - 1] - st[a]) / (b - a) / 1e3, 3)})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
