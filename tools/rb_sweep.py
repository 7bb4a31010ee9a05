#!/usr/bin/env python3
"""Row-block layout sweep on one matrix: HIP-event-timed SDDMM (warm, back-to-back launches) for
each tuning setting given as ENV=VALUE[,ENV=VALUE] strings; one JSON line per setting.

    python3 tools/rb_sweep.py --workload mycielskian15 --K 512 --alpha 0.5 --delta 0.3 \\
        --set "" --set BSMR_RB_ROWS=48 --set BSMR_RB_ROWS=80,BSMR_OUT_STAGED=0
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sddmm-gpu_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", required=True)
    ap.add_argument("--K", type=int, default=512)
    ap.add_argument("--alpha", type=float, default=0.3)
    ap.add_argument("--delta", type=float, default=0.3)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--set", action="append", default=[])
    args = ap.parse_args()
    import torch

    import bsmr
    from bsmr import Plan, make_data, synth, tuning_from_env

    M, N, rp, ci = synth.SUITESPARSE_REBUILDS[args.workload]()
    K = args.K
    dA = torch.from_numpy(make_data(M * K)).cuda()
    dB = torch.from_numpy(make_data(N * K)).cuda()
    dP = torch.zeros(len(ci), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream()
    for st in args.set or [""]:
        env = {k: v for k, v in os.environ.items() if k.startswith("BSMR_")}  # e.g. BSMR_DIAG
        env.update(kv.split("=", 1) for kv in st.split(",") if kv)
        plan = Plan(M, N, rp, ci, alpha=args.alpha, delta=args.delta, layout="rowblock",
                    tuning=tuning_from_env(env))
        run = lambda: plan.sddmm(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(),
                                 stream=s.cuda_stream, dtype=bsmr.F32)
        for _ in range(5):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(args.iters):
            run()
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        stats = plan.stats()
        print(json.dumps({"workload": args.workload, "K": K, "alpha": args.alpha,
                          "delta": args.delta, "set": st, "us": round(ms * 1e3, 2),
                          "gflops": round(2.0 * len(ci) * K / (ms * 1e6), 1),
                          "rb_rows": stats["rb_rows"], "rb_items": stats["rb_items"]}), flush=True)
        del plan


if __name__ == "__main__":
    main()
