#!/usr/bin/env python3
"""Per-kernel summary (calls, total / average / min / max duration in us) of a rocprofv3 run that
wrote its default SQLite output (rocpd `*_results.db`), as the `--stats` kernel table.

    python3 tools/rocpd_summary.py gpurun_out/<tag>/prof/prof_results.db > profiles/<tag>_kernel_stats.txt
"""
import sqlite3
import sys


def main(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), "
                     "max(duration) from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1.0
    print("calls\ttotal_us\tavg_us\tmin_us\tmax_us\tpct\tkernel")
    for name, n, tot, avg, mn, mx in rows:
        short = name if len(name) < 140 else name[:137] + "..."
        print(f"{n}\t{tot / 1e3:.3f}\t{avg / 1e3:.3f}\t{mn / 1e3:.3f}\t{mx / 1e3:.3f}\t"
              f"{100.0 * tot / total:.2f}\t{short}")


if __name__ == "__main__":
    main(sys.argv[1])
