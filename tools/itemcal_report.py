#!/usr/bin/env python3
"""Table of per-item timelines written by tools/item_trace.py (<dir>/*.npz): items, the ideal
span (sum of item durations / workgroup slots), the longest item, the measured span, and the
per-XCD busy time / end of the launch."""
import glob
import os
import sys

import numpy as np


def main(d):
    for f in sorted(glob.glob(os.path.join(d, "*.npz"))):
        n = os.path.basename(f)[:-4]
        z = np.load(f)
        RB, NT, nit, rowB, K, M, N, nnz = (int(v) for v in z["meta"])
        w = z["entries"] > 0
        du, st, x = z["dur_us"], z["start_us"], z["xcc"]
        slots = 256 * (2 if NT == 512 else 1)
        end = (st + du)[w].max()
        busy = [du[w & (x == X)].sum() / (slots // 8) for X in range(8)]
        print(f"{n:18s} RB={RB:4d} NT={NT:4d} items={int(w.sum()):6d} ideal={du[w].sum() / slots:8.1f} "
              f"max_item={du[w].max():7.1f} span={end:7.1f} TFLOP/s={2 * nnz * K / end / 1e6:6.1f} "
              f"xcd_busy=[{min(busy):.0f}..{max(busy):.0f}]")


if __name__ == "__main__":
    main(sys.argv[1])
