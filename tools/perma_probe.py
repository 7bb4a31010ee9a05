#!/usr/bin/env python3
"""Probe: does staging A from a copy already in reordered row order (contiguous row blocks)
beat staging the scattered rows of A? Times bsmr_sddmm (A in original order, staged through
reorderedRows) against bsmr_sddmm_panels_local over all panels (A_perm = A[reorderedRows],
staged through the identity), plus the cost of building A_perm on the device.

    python3 tools/perma_probe.py --workload reddit_like --scale 0.5
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sddmm-gpu_amd"))


def timed(fn, iters):
    import torch
    s = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="reddit_like")
    ap.add_argument("--scale", type=float, default=0.5)
    ap.add_argument("--K", type=int, default=128)
    ap.add_argument("--iters", type=int, default=30)
    args = ap.parse_args()
    import torch

    from bsmr import Plan, make_data, synth

    gen = getattr(synth, args.workload)
    M, N, rp, ci = gen(args.scale) if args.workload == "reddit_like" else gen()
    K = args.K
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3)
    P = plan.stats()["num_row_panels"]
    dA = torch.from_numpy(make_data(M * K)).cuda()
    dB = torch.from_numpy(make_data(N * K)).cuda()
    dP = torch.zeros(len(ci), dtype=torch.float32, device="cuda")
    rows = torch.from_numpy(plan.array("reorderedRows").astype("int64")).cuda()
    A2 = dA.view(M, K)
    Ap = A2.index_select(0, rows).contiguous()
    sp = torch.cuda.current_stream().cuda_stream
    out = {"M": M, "nnz": len(ci), "K": K}
    out["sddmm_ms"] = timed(lambda: plan.sddmm(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(),
                                               stream=sp), args.iters)
    P1 = dP.clone()
    out["panels_local_permuted_A_ms"] = timed(
        lambda: plan.sddmm_panels_local(Ap.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), 0, P,
                                        stream=sp), args.iters)
    out["same_values"] = bool(torch.allclose(P1, dP, rtol=1e-5, atol=1e-5))
    out["permute_A_ms"] = timed(lambda: torch.index_select(A2, 0, rows, out=Ap), args.iters)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
