#!/usr/bin/env python3
"""Offline study of a range-synchronised row-block sweep for the staged C4 layout (no GPU).

Per XCD x (column share cut into m ranges of equal entry count) every row block is a task run by
one of W workgroups (one per CU) that keeps the block's A image in LDS and walks the XCD's m
ranges in order; a workgroup may start range step g = r m + k (round r, range k) only once every
workgroup of the XCD has finished step g - s - 1 (slack s), so the B lines of at most s + 1
ranges are live in the XCD's L2 at a time. The tasks are dealt into rounds of W by descending
cost. Cost of a (row block, range) step = entries + piece_weight x column-run pieces (pieces cut
every 16 entries, the layout's cost model). Reports the sweep's makespan against the ideal
(total cost / W) per XCD, i.e. how much the per-step waits cost.

    python3 tools/sweep_sim.py --rows gpurun_out/r04v/rows_reddit_x1.npy --m 8 --slack 1
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sddmm-gpu_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", required=True)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--rb", type=int, default=240)
    ap.add_argument("--m", type=int, default=8, help="ranges per XCD")
    ap.add_argument("--slack", type=int, default=1)
    ap.add_argument("--wgs", type=int, default=32, help="workgroups per XCD")
    ap.add_argument("--piece-weight", type=float, default=4.0)
    ap.add_argument("--split", type=float, default=0.0,
                    help="split row blocks into tasks of at most this multiple of the mean cost")
    args = ap.parse_args()
    import numpy as np

    from bsmr import synth

    M, N, rp, ci = synth.reddit_like(args.scale)
    rp = np.asarray(rp, dtype=np.int64)
    ci = np.asarray(ci, dtype=np.int64)
    rows = np.load(args.rows).astype(np.int64)
    X = 8
    ncr = X * args.m
    # equal-entry column cuts
    colcnt = np.bincount(ci, minlength=N)
    cum = np.cumsum(colcnt)
    cuts = np.searchsorted(cum, np.arange(1, ncr) * cum[-1] / ncr)
    rng_of = np.zeros(N, dtype=np.int64)
    rng_of[cuts] += 1
    rng_of = np.cumsum(rng_of)
    nrb = (len(rows) + args.rb - 1) // args.rb
    cost = np.zeros((nrb, ncr))
    ent = np.zeros((nrb, ncr))
    pcs = np.zeros((nrb, ncr))
    for b in range(nrb):
        rr = rows[b * args.rb:(b + 1) * args.rb]
        cols = np.concatenate([ci[rp[r]:rp[r + 1]] for r in rr]) if len(rr) else np.zeros(0, np.int64)
        if cols.size == 0:
            continue
        u, cnt = np.unique(cols, return_counts=True)
        k = rng_of[u]
        e = np.bincount(k, weights=cnt, minlength=ncr)
        p = np.bincount(k, weights=np.ceil(cnt / 16.0), minlength=ncr)
        ent[b] = e
        pcs[b] = p
        cost[b] = e + args.piece_weight * p
    res = {"rows": int(len(rows)), "row_blocks": int(nrb), "m": args.m, "slack": args.slack,
           "wgs_per_xcd": args.wgs, "pieces_total": float(pcs.sum()),
           "entries_per_piece": float(ent.sum() / max(pcs.sum(), 1)), "xcd": []}
    W = args.wgs
    for x in range(X):
        c = cost[:, x * args.m:(x + 1) * args.m]  # task b: its m steps
        if args.split > 0:
            # heavy row blocks as several tasks (each stages the image and takes 1/h of every
            # range's entries): no task above split x the mean task cost
            tot = c.sum(1)
            h = np.maximum(1, np.ceil(tot / (args.split * tot.mean()))).astype(np.int64)
            c = np.repeat(c / h[:, None], h, axis=0)
        order = np.argsort(-c.sum(1), kind="stable")
        rounds = [order[i:i + W] for i in range(0, len(order), W)]
        steps = len(rounds) * args.m
        done = np.zeros(steps)  # time when every workgroup finished step g
        t = np.zeros(W)
        for r, tasks in enumerate(rounds):
            # the round's tasks (heaviest first) to the workgroups that are free earliest
            free = np.argsort(t, kind="stable")
            mine = np.full(W, -1)
            mine[free[:len(tasks)]] = tasks
            for k in range(args.m):
                g = r * args.m + k
                gate = done[g - args.slack - 1] if g - args.slack - 1 >= 0 else 0.0
                for w in range(W):
                    cw = c[mine[w], k] if mine[w] >= 0 else 0.0
                    t[w] = max(t[w], gate) + cw
                done[g] = t.max()
        ideal = c.sum() / W
        res["xcd"].append({"makespan": float(t.max()), "ideal": float(ideal),
                           "efficiency": float(ideal / t.max()), "tasks": int(len(c))})
    res["efficiency_min"] = min(v["efficiency"] for v in res["xcd"])
    res["efficiency_mean"] = float(np.mean([v["efficiency"] for v in res["xcd"]]))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
