#!/usr/bin/env python3
"""In-process A/B of launch layouts: one plan per tuning variant of the same pattern, each one's
steps captured into a HIP graph (as bench.py times them), the variants replayed in alternation for
several rounds; per variant the median µs per step and every round's value. One process and one
box for all variants, so clocks and box-to-box spread cancel.

    python3 tools/layout_ab.py --config C2 --variant rows:col_blocks=0 --variant cols: \\
        --variant split:col_blocks=1,diag=4096 --rounds 7
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sddmm-gpu_amd"))


def parse_variant(v):
    name, _, rest = v.partition(":")
    tun = {}
    for kv in filter(None, rest.split(",")):
        k, _, x = kv.partition("=")
        tun[k] = float(x) if "." in x else int(x)
    return name, tun


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2", choices=["C2", "C3", "C4", "C5u", "C5b"])
    ap.add_argument("--scale", type=float, default=0.25, help="C4 reddit-like size factor")
    ap.add_argument("--K", type=int, default=0)
    ap.add_argument("--variant", action="append", required=True, help="name:knob=v,knob=v")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--prespin-ms", type=float, default=0.0)
    ap.add_argument("--prespin-kind", default="sleep", choices=["sleep", "mm"])
    args = ap.parse_args()
    import torch

    from bsmr import BF16, F16, F32, Plan, make_data, synth

    if args.config == "C2":
        (M, N, rp, ci), K, dt = synth.nips_like(), args.K or 128, F32
    elif args.config == "C3":
        (M, N, rp, ci), K, dt = synth.cop20k_like(), args.K or 256, F16
    elif args.config == "C4":
        (M, N, rp, ci), K, dt = synth.reddit_like(args.scale), args.K or 128, F32
    else:
        (M, N, rp, ci), K, dt = synth.dlmc_like("uniform" if args.config == "C5u" else "block"), args.K or 512, BF16
    tdt = {F32: torch.float32, F16: torch.float16, BF16: torch.bfloat16}[dt]
    dev = torch.device("cuda", 0)
    dA = torch.from_numpy(make_data(M * K)).to(dev).to(tdt)
    dB = torch.from_numpy(make_data(N * K)).to(dev).to(tdt)
    dP = torch.zeros(len(ci), dtype=torch.float32, device=dev)
    gs = torch.cuda.Stream(dev)
    graphs, stats, mism, ref_P = {}, {}, {}, None
    for v in args.variant:
        name, tun = parse_variant(v)
        plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, tuning=tun)
        with torch.cuda.stream(gs):
            plan.sddmm(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), stream=gs.cuda_stream, dtype=dt)
        gs.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(gs):
            with torch.cuda.graph(g, stream=gs):
                for _ in range(args.steps):
                    plan.sddmm(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), stream=gs.cuda_stream, dtype=dt)
            g.replay()
        gs.synchronize()
        graphs[name] = (g, plan)
        Pv = dP.cpu().numpy().copy()
        if ref_P is None:
            ref_P = Pv
        else:  # the same products: checkData's rule against the first variant
            import numpy as np
            d = np.abs(Pv - ref_P)
            bad = (d >= 1e-5) & (d / np.maximum(np.maximum(np.abs(Pv), np.abs(ref_P)), 1e-3) >= 1e-3)
            mism[name] = int(bad.sum())
        st = plan.stats()
        stats[name] = {"tuning": tun, "rb_rows": st["rb_rows"], "rb_pieces": st["rb_pieces"],
                       "rb_col_blocks": st["rb_col_blocks"]}
    res = {k: [] for k in graphs}
    if args.prespin_ms > 0:  # device busy before the rounds: a spin, or real matmuls ("mm")
        with torch.cuda.stream(gs):
            if args.prespin_kind == "mm":
                x = torch.randn(4096, 4096, device=dev)
                t0 = torch.cuda.Event(enable_timing=True)
                t1 = torch.cuda.Event(enable_timing=True)
                t0.record(gs)
                for _ in range(int(args.prespin_ms / 0.06)):
                    x = x @ x
                    x = x / x.abs().max()
                t1.record(gs)
            else:
                torch.cuda._sleep(int(args.prespin_ms * 2.1e6))
        gs.synchronize()
    for _ in range(args.rounds):
        for name, (g, _) in graphs.items():
            with torch.cuda.stream(gs):
                torch.cuda._sleep(200_000)
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(gs)
                g.replay()
                e1.record(gs)
            gs.synchronize()
            res[name].append(round(e0.elapsed_time(e1) * 1e3 / args.steps, 3))
    out = {"config": args.config, "K": K, "steps": args.steps, "rounds": args.rounds,
           "median_us": {k: statistics.median(v) for k, v in res.items()}, "us": res, "layouts": stats,
           "checkData_errors_vs_first": mism}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
