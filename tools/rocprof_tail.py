#!/usr/bin/env python3
"""Per-dispatch view of the last N launches of one kernel in a rocprofv3 kernel trace: mean
duration, mean start-to-start interval and (span of the N launches) / N, i.e. what a timed
region of N back-to-back steps measures. bench.py's order is warm-up, stream-launched steps,
the graph's warm-up replay, then the timed graph replay, so the last `steps` dispatches of the
row-block kernel are the line's timed steps.

    python3 tools/rocprof_tail.py <run_kernel_trace.csv> [--kernel k_sddmm_rb] [--last 200]
"""
import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="k_sddmm_rb")
    ap.add_argument("--last", type=int, default=200)
    args = ap.parse_args()
    rows = [r for r in csv.DictReader(open(args.trace)) if args.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    out = {"kernel_dispatches": len(rows)}
    for name, sel in (("last", rows[-args.last:]), ("previous", rows[-2 * args.last:-args.last])):
        if len(sel) < 2:
            continue
        st = [int(r["Start_Timestamp"]) for r in sel]
        en = [int(r["End_Timestamp"]) for r in sel]
        dur = [e - s for s, e in zip(st, en)]
        gaps = [b - a for a, b in zip(st, st[1:])]
        out[name] = {"n": len(sel), "mean_duration_us": round(statistics.mean(dur) / 1e3, 3),
                     "median_duration_us": round(statistics.median(dur) / 1e3, 3),
                     "mean_start_to_start_us": round(statistics.mean(gaps) / 1e3, 3),
                     "span_per_launch_us": round((en[-1] - st[0]) / len(sel) / 1e3, 3)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
