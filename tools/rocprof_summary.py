#!/usr/bin/env python3
"""Summarise a rocprofv3 output directory (SQLite .db, or kernel_stats.csv) into a small text
table: kernel, calls, total us, average us, percent. Used to produce profiles/*.txt."""
import csv
import glob
import os
import sqlite3
import sys


def short(name, n=110):
    return name if len(name) <= n else name[: n - 3] + "..."


def from_db(path):
    c = sqlite3.connect(path)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage "
                          "from top_kernels"))
    # durations in the view are in microseconds? rocpd stores ns; the view reports ns/1000
    return rows


def from_csv(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3,
                         float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
    return rows


def main():
    d = sys.argv[1]
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    csvs = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    rows = from_csv(csvs[0]) if csvs else from_db(dbs[0])
    print(f"{'kernel':112s} {'calls':>6s} {'total_us':>12s} {'avg_us':>10s} {'pct':>6s}")
    for name, calls, tot, avg, pct in rows:
        print(f"{short(name):112s} {calls:6d} {tot:12.3f} {avg:10.3f} {pct:6.2f}")


if __name__ == "__main__":
    main()
