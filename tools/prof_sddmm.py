#!/usr/bin/env python3
"""Profiling driver: build the bench workload's plan once, then run the SDDMM kernel in its three
forms (dense-tile items only, residual items only, fused) `iters` times each through
bsmr_sddmm_profile, so rocprofv3 counter passes see only the launches of interest.

    rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_sddmm --output-format csv \
        -d gpurun_out/pmc_fetch -- python3 tools/prof_sddmm.py --iters 20
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sddmm-gpu_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--K", type=int, default=128)
    ap.add_argument("--workload", default="nips_like")
    ap.add_argument("--layout", default="auto", choices=["auto", "rowblock", "colmajor"])
    ap.add_argument("--lds-kb", type=int, default=0)
    ap.add_argument("--dtype", default="f32", choices=["f32", "f16", "bf16"])
    ap.add_argument("--scale", type=float, default=None, help="reddit_like size factor")
    ap.add_argument("--mask", default=None, help="dlmc_like mask: uniform | block")
    ap.add_argument("--diag", type=int, default=0, help="BSMR_DIAG ablation bits (sddmm.hip)")
    ap.add_argument("--alpha", type=float, default=0.3)
    ap.add_argument("--delta", type=float, default=0.3)
    args = ap.parse_args()
    if args.diag:
        os.environ["BSMR_DIAG"] = str(args.diag)
    import torch

    import bsmr
    from bsmr import Plan, make_data, set_default_tuning, synth, tuning_from_env

    if args.workload in synth.SUITESPARSE_REBUILDS:  # e.g. Trefethen_20000, mycielskian15
        gen = synth.SUITESPARSE_REBUILDS[args.workload]
    else:
        gen = getattr(synth, args.workload)
    if args.mask is not None:
        M, N, rp, ci = gen(args.mask)
    else:
        M, N, rp, ci = gen(args.scale) if args.scale is not None else gen()
    K = args.K
    set_default_tuning(tuning_from_env())  # BSMR_* A/B knobs (the library reads no env)
    plan = Plan(M, N, rp, ci, alpha=args.alpha, delta=args.delta, layout=args.layout,
                lds_budget_kb=args.lds_kb)
    tdt = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}[args.dtype]
    code = {"f32": bsmr.F32, "f16": bsmr.F16, "bf16": bsmr.BF16}[args.dtype]
    dA = torch.from_numpy(make_data(M * K)).cuda().to(tdt)
    dB = torch.from_numpy(make_data(N * K)).cuda().to(tdt)
    dP = torch.zeros(len(ci), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    plan.sddmm(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), stream=s, dtype=code)
    r = plan.profile(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), iters=args.iters, stream=s,
                     dtype=code)
    torch.cuda.synchronize()
    st = plan.stats()
    print(json.dumps({"M": M, "N": N, "nnz": len(ci), "K": K, "dtype": args.dtype,
                      "workload": args.workload, "layout": args.layout,
                      "rb": {k: st[k] for k in ("rb_rows", "rb_items", "rb_pieces", "rb_work_items",
                                                "rb_orig_rows")},
                      "lds_kb": args.lds_kb, "timing_ms": r,
                      "dense_items": st["dense_items"], "residual_slots_hint": st["residual_items"],
                      "dense_tiles": st["num_dense_tiles"], "residual": st["num_residual"]}))


if __name__ == "__main__":
    main()
