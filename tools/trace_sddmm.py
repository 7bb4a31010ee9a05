#!/usr/bin/env python3
"""Wave timeline of one SDDMM launch (debug build switch BSMR_DIAG=32, set by this script before
the plan is created): per wave start / mid / end (s_memrealtime, 100 MHz) and hardware ids.
Prints percentiles of dispatch time, wave lifetime and end time, overall and per XCD."""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sddmm-gpu_amd"))


def pct(x):
    if len(x) == 0:
        return None
    return [round(float(v), 3) for v in np.percentile(x, [0, 10, 50, 90, 100])]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=128)
    ap.add_argument("--workload", default="nips_like")
    ap.add_argument("--layout", default="auto")
    ap.add_argument("--lds-kb", type=int, default=0)
    ap.add_argument("--dump", default="")
    ap.add_argument("--dtype", default="f32", choices=["f32", "f16", "bf16"])
    ap.add_argument("--scale", type=float, default=None, help="reddit_like size factor")
    ap.add_argument("--waves-per-wg", type=int, default=16, help="NT / 64 of the traced launch")
    ap.add_argument("--mask", default=None, help="dlmc_like mask: uniform | block")
    ap.add_argument("--cold", nargs="?", const="write", default=None, choices=["write", "read"],
                    help="trace a launch right after a 512 MiB write (Infinity Cache evicted, as "
                         "bench.py's cold leg), or after a 512 MiB read (--cold read: evicted, "
                         "caches clean, as the cold leg's 'clean' figure)")
    args = ap.parse_args()
    os.environ["BSMR_DIAG"] = str(int(os.environ.get("BSMR_DIAG", "0")) | 32)
    import torch

    import bsmr
    from bsmr import Plan, make_data, set_default_tuning, synth, tuning_from_env

    gen = getattr(synth, args.workload)
    if args.mask is not None:
        M, N, rp, ci = gen(args.mask)
    else:
        M, N, rp, ci = gen(args.scale) if args.scale is not None else gen()
    K = args.K
    set_default_tuning(tuning_from_env())  # BSMR_* A/B knobs (the library reads no env)
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, layout=args.layout, lds_budget_kb=args.lds_kb)
    tdt = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}[args.dtype]
    code = {"f32": bsmr.F32, "f16": bsmr.F16, "bf16": bsmr.BF16}[args.dtype]
    dA = torch.from_numpy(make_data(M * K)).cuda().to(tdt)
    dB = torch.from_numpy(make_data(N * K)).cuda().to(tdt)
    dP = torch.zeros(len(ci), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(10):
        plan.sddmm(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), stream=s, dtype=code)
    torch.cuda.synchronize()
    if args.cold:  # evict the MALL, then the traced launch
        flush = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
        flush.fill_(1)
        if args.cold == "read":
            sink = torch.empty((), dtype=torch.int64, device="cuda")
            for _ in range(3):
                sink.copy_(flush.sum(dtype=torch.int64))
        torch.cuda.synchronize()
        plan.sddmm(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), stream=s, dtype=code)
        torch.cuda.synchronize()
    L = bsmr.lib()
    L.bsmr_debug_trace.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64)]
    n = C.c_uint64()
    L.bsmr_debug_trace(plan.h, None, C.byref(n))
    buf = np.zeros(n.value, np.uint64)
    L.bsmr_debug_trace(plan.h, buf.ctypes.data, C.byref(n))
    t = buf.reshape(-1, 4)
    slot = np.arange(len(t))
    keep = t[:, 2] > 0
    t, slot = t[keep], slot[keep]
    if args.dump:
        np.save(args.dump, t)
    t0, tm, t1 = (t[:, i].astype(np.int64) for i in range(3))
    td = (t[:, 3] & np.uint64((1 << 60) - 1)).astype(np.int64)
    base = t0.min()
    us = 0.01  # 100 MHz ticks -> us
    xcc = (t[:, 3] >> np.uint64(60)).astype(np.int64) & 0xF
    out = {"K": K, "workload": args.workload, "dtype": args.dtype, "layout": args.layout,
           "cold": args.cold,
           "lds_kb": args.lds_kb, "waves": int(len(t)),
           "rb": {k: plan.stats()[k] for k in ("rb_rows", "rb_items", "rb_pieces")},
           "span_us": round(float((t1.max() - base) * us), 3),
           "start_us": pct((t0 - base) * us), "life_us": pct((t1 - t0) * us),
           "mid_us": pct((tm - t0) * us), "dense_us": pct((td - tm) * us),
           "tail_us": pct((t1 - td) * us), "end_us": pct((t1 - base) * us),
           "per_xcd": {},
           # workgroup b = slot // waves-per-wg; the layout assumes XCD = b % 8
           "xcd_is_block_mod8": float(np.mean(xcc == (slot // args.waves_per_wg) % 8))}
    for x in range(8):
        m = xcc == x
        if m.any():
            out["per_xcd"][x] = {"waves": int(m.sum()), "start_p50": float(np.median(t0[m] - base) * us),
                                 "end_max": float((t1[m].max() - base) * us)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
