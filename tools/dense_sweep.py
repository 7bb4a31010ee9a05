#!/usr/bin/env python3
"""Dense-sampled vs gathered launch for fp16/bf16 uniform masks over a density sweep (the
crossover that sets Plan::dense_min): per density, TFLOP/s (2 nnz K / time) of the layout-auto
launch with BSMR_DENSE_MIN = 0 (dense-sampled) and = 2 (row-block / column-major).

    python3 tools/dense_sweep.py --n 2048 --K 512 --densities 0.005,0.01,0.02,0.05,0.1
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sddmm-gpu_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--K", type=int, default=512)
    ap.add_argument("--dtype", default="bf16", choices=["f16", "bf16"])
    ap.add_argument("--densities", default="0.005,0.01,0.02,0.03,0.05,0.1")
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    import torch

    import bsmr
    from bsmr import Plan, make_data, synth, tuning_from_env

    code = bsmr.BF16 if args.dtype == "bf16" else bsmr.F16
    tdt = torch.bfloat16 if args.dtype == "bf16" else torch.float16
    K, n = args.K, args.n
    dA = torch.from_numpy(make_data(n * K)).cuda().to(tdt)
    dB = torch.from_numpy(make_data(n * K)).cuda().to(tdt)
    s = torch.cuda.current_stream()
    out = {"n": n, "K": K, "dtype": args.dtype, "runs": []}
    for d in [float(x) for x in args.densities.split(",")]:
        M, N, rp, ci = synth.uniform_mask(n, d, seed=7)
        row = {"density": d, "nnz": len(ci)}
        res = {}
        for name, env in (("dense", "0"), ("gather", "2")):
            os.environ["BSMR_DENSE_MIN"] = env  # read at plan creation
            plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, tuning=tuning_from_env())
            dP = torch.zeros(len(ci), dtype=torch.float32, device="cuda")
            call = lambda: plan.sddmm(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(),  # noqa: E731
                                      stream=s.cuda_stream, dtype=code)
            for _ in range(3):
                call()
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(args.iters):
                call()
            e1.record(s)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.iters
            res[name] = dP.cpu().numpy()
            row[name] = {"us": round(ms * 1e3, 2),
                         "TFLOP/s": round(2.0 * len(ci) * K / (ms * 1e-3) / 1e12, 2)}
            del plan
        diff = float(abs(res["dense"] - res["gather"]).max())
        row["max_abs_diff"] = diff
        out["runs"].append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)
    os.environ.pop("BSMR_DENSE_MIN", None)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
