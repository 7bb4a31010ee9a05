#!/usr/bin/env python3
"""A/B: the C2 launch against the same products computed on the transposed pattern.

P[i, j] = A_i . B_j is symmetric in the roles of A and B: a row-block launch over S^T stages B
rows (S's columns) in LDS and gathers A rows per column-run piece. On a wide pattern (C2: 1,500 x
12,419) the column blocks are longer in stored entries per gathered row than the row blocks
(offline count, 256-row / 256-column blocks: 95.5 K pieces against 83.6 K). This times both —
the plan of S (the product launch) and a plan of S^T with A and B swapped (its P in S^T's CSR
order, so only the time is compared) — alternating, 200 launches per timing, HIP events.
Caveat (round 6): the variants run in a fixed order each round, so the first one also carries the
device's ramp from a standing start; tools/layout_ab.py (graphs, many rounds) is the A/B to trust —
on it the column-block layout (col_blocks = 1) times the same as the row-block one.

    python3 tools/transpose_ab.py [--reps 3] [--orig -1|0|1]
"""
import argparse
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sddmm-gpu_amd"))


def transpose(M, N, rp, ci):
    rp = np.asarray(rp, np.int64)
    ci = np.asarray(ci, np.int64)
    rows = np.repeat(np.arange(M, dtype=np.int64), np.diff(rp))
    order = np.lexsort((rows, ci))
    cp = np.zeros(N + 1, np.int64)
    np.cumsum(np.bincount(ci, minlength=N), out=cp[1:])
    return N, M, cp.astype(np.uint32), rows[order].astype(np.uint32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--K", type=int, default=128)
    ap.add_argument("--rb-rows", type=int, nargs="*", default=[128, 256, 304],
                    help="forced rows per block of the S^T launch (besides its own rule, -1)")
    ap.add_argument("--s-rb-rows", type=int, nargs="*", default=[],
                    help="forced rows per block of extra S launches (original and BSMR row order)")
    args = ap.parse_args()
    import torch

    from bsmr import Plan, make_data, synth

    M, N, rp, ci = synth.nips_like()
    K = args.K
    Mt, Nt, rpt, cit = transpose(M, N, rp, ci)
    dev = torch.device("cuda", 0)
    dA = torch.from_numpy(make_data(M * K)).to(dev)
    dB = torch.from_numpy(make_data(N * K)).to(dev)
    dP = torch.zeros(len(ci), dtype=torch.float32, device=dev)
    s = torch.cuda.current_stream(dev)
    plans = {"S": (Plan(M, N, rp, ci, alpha=0.3, delta=0.3), dA, dB),
             "S_rows": (Plan(M, N, rp, ci, alpha=0.3, delta=0.3, tuning={"col_blocks": 0}), dA, dB)}
    for orig in (0, 1):
        for rbr in args.s_rb_rows:
            plans[f"S_orig{orig}_rb{rbr}"] = (Plan(M, N, rp, ci, alpha=0.3, delta=0.3,
                                                   tuning={"orig_rows": orig, "rb_rows": rbr}), dA, dB)
    for orig in (0, 1):
        for rbr in [-1] + args.rb_rows:
            plans[f"ST_orig{orig}_rb{rbr}"] = (Plan(Mt, Nt, rpt, cit, alpha=0.3, delta=0.3,
                                                    tuning={"orig_rows": orig, "rb_rows": rbr}), dB, dA)

    def timed(name):
        plan, X, Y = plans[name]
        for _ in range(3):
            plan.sddmm(X.data_ptr(), Y.data_ptr(), K, dP.data_ptr(), stream=s.cuda_stream)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(args.steps):
            plan.sddmm(X.data_ptr(), Y.data_ptr(), K, dP.data_ptr(), stream=s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / args.steps

    res = {k: [] for k in plans}
    for _ in range(args.reps):
        for k in plans:
            res[k].append(timed(k))
    out = {"workload": f"C2 nips_like fp32 K={K}", "us_per_launch": {k: [round(x, 3) for x in v] for k, v in res.items()},
           "median_us": {k: round(statistics.median(v), 3) for k, v in res.items()}}
    for k, (plan, _, _) in plans.items():
        st = plan.stats()
        out[f"layout_{k}"] = {f: st[f] for f in ("rb_rows", "rb_items", "rb_pieces", "num_dense_tiles",
                                                  "num_residual")}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
