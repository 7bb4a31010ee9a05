#!/usr/bin/env python3
"""Wave balance of the row-block launch's piece dealing, from the layout itself (GPU: the plan and
its layout are built on the device; the model runs on the host).

A wave runs its 64 / G row-groups in lockstep, so in each phase it takes as long as its longest
piece (entries; + a per-piece cost for the B gather). Per item, this prints the wave times of the
static dealing (phase ph: pieces [ph NG, (ph + 1) NG), forwards in even and backwards in odd
phases) and of dynamic batches (wave w takes batch w, then the next batch from a counter), as the
item span (the slowest wave) against the mean wave, and the launch's item spans.

    python3 tools/phase_balance.py --workload nips_like --K 128
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sddmm-gpu_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="nips_like")
    ap.add_argument("--scale", type=float, default=None)
    ap.add_argument("--K", type=int, default=128)
    ap.add_argument("--dtype", default="f32", choices=["f32", "f16", "bf16"])
    ap.add_argument("--piece-cost", type=float, default=4.0, help="entry-steps per piece (B gather)")
    args = ap.parse_args()
    import bsmr
    from bsmr import Plan, synth

    gen = getattr(synth, args.workload)
    M, N, rp, ci = gen(args.scale) if args.scale is not None else gen()
    code = {"f32": bsmr.F32, "f16": bsmr.F16, "bf16": bsmr.BF16}[args.dtype]
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3)
    L = bsmr.lib()
    L.bsmr_debug_rb_pieces.argtypes = [C.c_void_p, C.c_uint32, C.c_int, C.c_void_p, C.POINTER(C.c_uint64)]
    n = C.c_uint64()
    assert L.bsmr_debug_rb_pieces(plan.h, args.K, code, None, C.byref(n)) == 0
    buf = np.zeros(n.value, np.uint32)
    assert L.bsmr_debug_rb_pieces(plan.h, args.K, code, buf.ctypes.data, C.byref(n)) == 0
    ni, npc = int(buf[0]), int(buf[1])
    items = buf[2:2 + 4 * ni].reshape(-1, 4)
    ends = buf[2 + 4 * ni:2 + 5 * ni]
    pieces = buf[2 + 5 * ni:2 + 5 * ni + 2 * npc].reshape(-1, 2)
    plen = (pieces[:, 1] >> 22).astype(np.int64) + 1
    stats = plan.stats()
    slot = [i for i in range(5) if stats["rb_items"][i]][0]
    row_bytes = 128 << slot
    G = 16 if row_bytes >= 2048 else 8 if row_bytes >= 1024 else 4
    NT = 1024 if stats["rb_rows"][slot] * row_bytes > 80 * 1024 else 512
    NW, GW = NT // 64, 64 // G
    NG = NW * GW
    cost = lambda ls: (ls.max() + args.piece_cost) if len(ls) else 0.0  # noqa: E731
    spans_s, spans_d, means = [], [], []
    for i in range(ni):
        p0, p1 = int(items[i, 3]), int(ends[i])
        if p1 <= p0:
            continue
        ln = plen[p0:p1]
        np_ = len(ln)
        # static: group gr takes pieces ph NG + (gr | NG - 1 - gr)
        wave = np.zeros(NW)
        ph = 0
        while ph * NG < np_:
            for w in range(NW):
                gs = np.arange(w * GW, (w + 1) * GW)
                pi = ph * NG + (NG - 1 - gs if ph & 1 else gs)
                pi = pi[pi < np_]
                wave[w] += cost(ln[pi])
            ph += 1
        # dynamic: batch b = pieces [b GW, (b + 1) GW); wave w starts with batch w, then takes the
        # next batch when it is free (event order)
        nb = (np_ + GW - 1) // GW
        bcost = np.array([cost(ln[b * GW:(b + 1) * GW]) for b in range(nb)])
        t = np.zeros(NW)
        for w in range(min(NW, nb)):
            t[w] = bcost[w]
        for b in range(NW, nb):
            w = int(np.argmin(t))
            t[w] += bcost[b]
        spans_s.append(wave.max())
        spans_d.append(t.max())
        means.append(bcost.sum() / NW)
    spans_s, spans_d, means = map(np.array, (spans_s, spans_d, means))
    out = {"workload": args.workload, "K": args.K, "items": int(len(means)), "pieces": npc,
           "row_bytes": row_bytes, "NT": NT, "pieces_per_rowgroup": round(npc / len(means) / NG, 2),
           "static_span_over_mean_p50": round(float(np.median(spans_s / means)), 3),
           "dynamic_span_over_mean_p50": round(float(np.median(spans_d / means)), 3),
           "static_launch_max": round(float(spans_s.max()), 1), "dynamic_launch_max": round(float(spans_d.max()), 1),
           "mean_wave_max": round(float(means.max()), 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
