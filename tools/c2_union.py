#!/usr/bin/env python3
"""Per-item union of kept-tile B columns on C2 ("commit the per-item
union-size histogram first").

The C2 launch (nips_like, fp32 K = 128) runs 256 row-block items: a 256-row image of A in LDS
(128 KiB of the 160) and one column range of the pattern each. Keeping the plan's 16 x 16 tiles on
MFMA inside such an item would read each tile's 16 B columns; staging the union of those columns
once per item into the LDS left next to the image would serve the tiles and the same columns'
column-run pieces from LDS. This counts, per item of the default layout, the distinct dense
(tile) columns of the item's panels that fall in its column range (the range spanned by its
pieces' columns), and the bytes they would take (512 per column), against the LDS the image leaves.

    python3 tools/c2_union.py > c2_union.json
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sddmm-gpu_amd"))


def main():
    import bsmr
    from bsmr import Plan, synth

    M, N, rp, ci = synth.nips_like()
    K = 128
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3)
    L = bsmr.lib()
    L.bsmr_debug_rb_items.argtypes = [C.c_void_p, C.c_uint32, C.c_int, C.c_void_p, C.POINTER(C.c_uint64)]
    L.bsmr_debug_rb_pieces.argtypes = [C.c_void_p, C.c_uint32, C.c_int, C.c_void_p, C.POINTER(C.c_uint64)]
    n = C.c_uint64()
    L.bsmr_debug_rb_items(plan.h, K, 0, None, C.byref(n))
    hdr = np.zeros(n.value, np.uint32)
    L.bsmr_debug_rb_items(plan.h, K, 0, hdr.ctypes.data, C.byref(n))
    RB, rowBytes = int(hdr[0]), int(hdr[3])
    L.bsmr_debug_rb_pieces(plan.h, K, 0, None, C.byref(n))
    buf = np.zeros(n.value, np.uint32)
    L.bsmr_debug_rb_pieces(plan.h, K, 0, buf.ctypes.data, C.byref(n))
    ni, npc = int(buf[0]), int(buf[1])
    items = buf[2:2 + 4 * ni].reshape(ni, 4)
    iend = buf[2 + 4 * ni:2 + 5 * ni]
    pieces = buf[2 + 5 * ni:2 + 5 * ni + 2 * npc].reshape(npc, 2)
    pcol = pieces[:, 1] & 0x3FFFFF
    dco = plan.array("denseColOffsets").astype(np.int64)
    dcols = plan.array("denseCols").astype(np.int64)
    free = 160 * 1024 - RB * rowBytes
    unions, entries = [], []
    for i in range(ni):
        p0, p1 = int(items[i, 3]), int(iend[i])
        if p1 <= p0:
            continue
        lo, hi = int(pcol[p0:p1].min()), int(pcol[p0:p1].max())
        rb = int(items[i, 0])
        pn0, pn1 = rb * RB // 16, min((rb + 1) * RB // 16, len(dco) - 1)
        cols = dcols[dco[pn0]:dco[pn1]]
        cols = cols[(cols >= lo) & (cols <= hi) & (cols < N)]
        unions.append(len(np.unique(cols)))
        entries.append(p1 - p0)
    u = np.array(unions)
    out = {"workload": "C2 nips_like fp32 K=128", "rows_per_block": RB, "items": len(u),
           "image_bytes": RB * rowBytes, "free_lds_bytes": free,
           "free_lds_columns": free // rowBytes,
           "union_columns": {"p0": int(u.min()), "p25": int(np.percentile(u, 25)),
                             "p50": int(np.median(u)), "p75": int(np.percentile(u, 75)),
                             "p100": int(u.max()), "mean": round(float(u.mean()), 1)},
           "union_bytes_p50": int(np.median(u)) * rowBytes,
           "items_fitting": int((u * rowBytes <= free).sum()),
           "histogram_columns": {f"{int(a)}-{int(b) - 1}": int(c) for a, b, c in
                                 zip(*(lambda h: (h[1][:-1], h[1][1:], h[0]))(
                                     np.histogram(u, bins=[0, 32, 64, 128, 256, 512, 1024, 4096, 1 << 20])))}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
