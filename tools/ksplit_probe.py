#!/usr/bin/env python3
"""Probe for a K-split of graph SDDMMs: time the row-block launch of one plan at K = 32 / 64 /
128 / 256 (fp32; rows of 128 / 256 / 512 / 1024 B, so row blocks of 1024 / 576 / 288 / 144 rows)
and report the layout sizes. If S launches over K/S-wide slices beat one K-wide launch, a K-split
of the K-wide problem pays (longer column runs per row block).

    python3 tools/ksplit_probe.py --workload reddit_like --scale 0.5
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sddmm-gpu_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="reddit_like")
    ap.add_argument("--scale", type=float, default=0.5)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    import torch

    from bsmr import Plan, make_data, synth

    gen = getattr(synth, args.workload)
    M, N, rp, ci = gen(args.scale) if args.workload == "reddit_like" else gen()
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3)
    out = {"M": M, "N": N, "nnz": len(ci)}
    for K in (32, 64, 128, 256):
        dA = torch.from_numpy(make_data(M * K)).cuda()
        dB = torch.from_numpy(make_data(N * K)).cuda()
        dP = torch.zeros(len(ci), dtype=torch.float32, device="cuda")
        s = torch.cuda.current_stream()
        plan.sddmm(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), stream=s.cuda_stream)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(args.iters):
            plan.sddmm(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), stream=s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        st = plan.stats()
        i = {32: 0, 64: 1, 128: 2, 256: 3}[K]
        out[K] = {"ms": round(ms, 4), "TFLOPs": round(2 * len(ci) * K / ms / 1e9, 2),
                  "rb_rows": st["rb_rows"][i], "items": st["rb_items"][i],
                  "pieces": st["rb_pieces"][i]}
        print(json.dumps({K: out[K]}), flush=True)
        del dA, dB, dP
    print(json.dumps(out))


if __name__ == "__main__":
    main()
