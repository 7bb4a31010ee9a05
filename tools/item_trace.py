#!/usr/bin/env python3
"""Per-item timeline of one row-block launch, for calibrating the item cost model (plan.hip
build_rowblock_layout): the debug trace (BSMR_DIAG=32, per wave start / end, s_memrealtime at
100 MHz) folded per workgroup = item, joined with each item's layout stats (row block, kept tiles,
entries, column-run pieces; bsmr_debug_rb_items). Writes <out>.npz (columns below) and prints a
JSON summary line.

    python3 tools/item_trace.py --workload mycielskian15 --K 256 --alpha 0.5 --delta 0.7 \\
        --out gpurun_out/it/myc15_K256
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
    ap.add_argument("--alpha", type=float, default=0.3)
    ap.add_argument("--delta", type=float, default=0.3)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    os.environ["BSMR_DIAG"] = str(int(os.environ.get("BSMR_DIAG", "0")) | 32)
    import torch

    import bsmr
    from bsmr import Plan, make_data, set_default_tuning, synth, tuning_from_env

    if args.workload in synth.SUITESPARSE_REBUILDS:
        gen = synth.SUITESPARSE_REBUILDS[args.workload]
        M, N, rp, ci = gen()
    else:
        gen = getattr(synth, args.workload)
        M, N, rp, ci = gen(args.scale) if args.scale is not None else gen()
    set_default_tuning(tuning_from_env())
    plan = Plan(M, N, rp, ci, alpha=args.alpha, delta=args.delta, layout="rowblock")
    K = args.K
    tdt = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}[args.dtype]
    code = {"f32": bsmr.F32, "f16": bsmr.F16, "bf16": bsmr.BF16}[args.dtype]
    dA = torch.from_numpy(make_data(M * K)).cuda().to(tdt)
    dB = torch.from_numpy(make_data(N * K)).cuda().to(tdt)
    dP = torch.zeros(len(ci), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    L = bsmr.lib()
    L.bsmr_debug_trace.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64)]
    L.bsmr_debug_rb_items.argtypes = [C.c_void_p, C.c_uint32, C.c_int, C.c_void_p,
                                      C.POINTER(C.c_uint64)]
    spans, runs = [], []
    for _ in range(args.iters):  # keep the last launch's trace; the span of each
        plan.sddmm(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), stream=s, dtype=code)
        torch.cuda.synchronize()
        n = C.c_uint64()
        L.bsmr_debug_trace(plan.h, None, C.byref(n))
        buf = np.zeros(n.value, np.uint64)
        L.bsmr_debug_trace(plan.h, buf.ctypes.data, C.byref(n))
        runs.append(buf.reshape(-1, 4).copy())
    n = C.c_uint64()
    assert L.bsmr_debug_rb_items(plan.h, K, code, None, C.byref(n)) == 0
    it = np.zeros(n.value, np.uint32)
    assert L.bsmr_debug_rb_items(plan.h, K, code, it.ctypes.data, C.byref(n)) == 0
    RB, NT, nitems, rowBytes = (int(v) for v in it[:4])
    stat = it[4:].reshape(-1, 4).astype(np.int64)
    wpg = NT // 64
    per_item = []
    for t in runs:
        t = t[: nitems * wpg].reshape(nitems, wpg, 4)
        t0 = t[:, :, 0].astype(np.int64)
        t1 = t[:, :, 2].astype(np.int64)
        live = t1 > 0
        st = np.where(live, t0, np.iinfo(np.int64).max).min(axis=1)
        en = np.where(live, t1, 0).max(axis=1)
        base = st[live.any(axis=1)].min()
        ok = live.any(axis=1)
        spans.append(float((en[ok].max() - base) * 0.01))
        per_item.append((np.where(ok, (st - base) * 0.01, -1.0), np.where(ok, (en - st) * 0.01, -1.0)))
    start = np.median(np.stack([p[0] for p in per_item]), axis=0)
    dur = np.median(np.stack([p[1] for p in per_item]), axis=0)
    xcc = (runs[-1][: nitems * wpg].reshape(nitems, wpg, 4)[:, 0, 3] >> np.uint64(60)).astype(np.int64) & 0xF
    np.savez(args.out + ".npz", rb=stat[:, 0], tiles=stat[:, 1], entries=stat[:, 2],
             pieces=stat[:, 3], start_us=start, dur_us=dur, xcc=xcc,
             dur_all=np.stack([p[1] for p in per_item]), start_all=np.stack([p[0] for p in per_item]),
             meta=np.array([RB, NT, nitems, rowBytes, K, M, N, len(ci)], np.int64))
    work = stat[:, 2] > 0
    st = plan.stats()
    print(json.dumps({"workload": args.workload, "K": K, "dtype": args.dtype, "RB": RB, "NT": NT,
                      "items": nitems, "work_items": int(work.sum()), "rowBytes": rowBytes,
                      "span_us_p50": float(np.median(spans)),
                      "dur_us": [round(float(v), 2) for v in np.percentile(dur[work], [0, 50, 90, 100])],
                      "entries": int(stat[:, 2].sum()), "pieces": int(stat[:, 3].sum()),
                      "tiles": int(stat[:, 1].sum()), "rb_rows": st["rb_rows"]}))


if __name__ == "__main__":
    main()
