#!/usr/bin/env python3
"""Standing performance regression guard for the launch-layout rules.

Re-times a fixed set of points — the 20 published SuiteSparse points the reference's results
CSVs hold for the five matrices bsmr/synth.py rebuilds exactly (Trefethen_20000, Trefethen_20000b,
mycielskian14/15/16 at K = 32, 64, 128, 256; each at the (alpha, delta) its test-mode sweep found
best, rows 7 / 350 / 363 / 367 / 444 of scripts/results_suiteSparse_dataset/k*/results_*.csv) and
the bench configs C2 (K = 32 / 128 / 512), C3, C4 x0.5, C4 x1, C5 uniform / block — and compares
them with a committed baseline (profiles/perf_baseline.json). Any point more than --tol (5 %)
slower than the run's median slowdown (the box factor: boxes differ by a few percent), or a box
factor itself above --tol, fails the run (exit 1), so a layout rule fitted on a few matrices cannot silently slow a
published point again (round 4: the pair / range rules took mycielskian15 K = 64 from 16.1 to
12.6 TFLOP/s and were found only by a manual refresh).

Timing: plan built once per point, 3 warm-up launches, then 5 batches of `iters` back-to-back
launches between HIP events; the fastest batch is the point's ms per launch (the small points,
7-10 us kernels, show bimodal batch times within one run: r05s Trefethen_20000b K = 32 batches
7.38 / 8.26 / 7.97 us on an unchanged library; the minimum is what a layout change moves).

    python3 tools/perf_guard.py --record profiles/perf_baseline.json     # new baseline
    python3 tools/perf_guard.py --check profiles/perf_baseline.json      # guard (rc 1 on loss)
    BSMR_PIECE_MAX=4 python3 tools/perf_guard.py --check ...             # a bad knob trips it
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sddmm-gpu_amd"))

# (alpha, delta) of the best test-mode setting per (matrix, K) on MI355X
# (profiles/r04zv/ss_compare_8f76aec.json)
# (a copy of profiles/r04zv/ss_compare_8f76aec.json outside the round directories, which GPU runs
# do not receive: .gpurunignore)
SS_BEST_FILE = os.path.join(ROOT, "profiles", "perf_guard_ss_points.json")
SS = ["Trefethen_20000", "Trefethen_20000b", "mycielskian14", "mycielskian15", "mycielskian16"]


def points():
    best = json.load(open(SS_BEST_FILE))["matrices"]
    pts = []
    for m in SS:
        for K in (32, 64, 128, 256):
            v = best[m]["K"][str(K)]
            pts.append({"name": f"{m}_K{K}", "matrix": m, "K": K, "dtype": "f32",
                        "alpha": v["alpha"], "delta": v["delta"], "iters": 50})
    cfg = [("C2_K128", "nips_like", None, 128, "f32", 200), ("C2_K32", "nips_like", None, 32, "f32", 200),
           ("C2_K512", "nips_like", None, 512, "f32", 100), ("C3", "cop20k_like", None, 256, "f16", 100),
           ("C4_x0.5", "reddit_like", 0.5, 128, "f32", 10), ("C4_x1", "reddit_like", 1.0, 128, "f32", 5),
           ("C5_uniform", "dlmc_like", "uniform", 512, "bf16", 200),
           ("C5_block", "dlmc_like", "block", 512, "bf16", 200)]
    for name, gen, arg, K, dt, iters in cfg:
        pts.append({"name": name, "matrix": gen, "arg": arg, "K": K, "dtype": dt, "alpha": 0.3,
                    "delta": 0.3, "iters": iters})
    return pts


def pattern(p):
    from bsmr import synth

    if p["matrix"] in synth.SUITESPARSE_REBUILDS:
        return synth.SUITESPARSE_REBUILDS[p["matrix"]]()
    gen = getattr(synth, p["matrix"])
    return gen() if p.get("arg") is None else gen(p["arg"])


def time_point(p):
    import torch

    import bsmr
    from bsmr import Plan, make_data

    M, N, rp, ci = pattern(p)
    K = p["K"]
    code = {"f32": bsmr.F32, "f16": bsmr.F16, "bf16": bsmr.BF16}[p["dtype"]]
    tdt = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}[p["dtype"]]
    plan = Plan(M, N, rp, ci, alpha=p["alpha"], delta=p["delta"])
    dA = torch.from_numpy(make_data(M * K)).cuda().to(tdt)
    dB = torch.from_numpy(make_data(N * K)).cuda().to(tdt)
    dP = torch.zeros(len(ci), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream()

    def launch():
        plan.sddmm(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), stream=s.cuda_stream, dtype=code)

    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    batches = []
    for _ in range(5):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(p["iters"]):
            launch()
        e1.record(s)
        torch.cuda.synchronize()
        batches.append(e0.elapsed_time(e1) / p["iters"])
    ms = min(batches)
    st = plan.stats()
    del plan, dA, dB, dP
    return {"ms": round(ms, 5), "gflops": round(2.0 * len(ci) * K / (ms * 1e-3) / 1e9, 1),
            "batches_ms": [round(b, 5) for b in batches],
            "rb_items": max(st["rb_items"]), "rb_pieces": max(st["rb_pieces"]),
            "rb_pairs": st["rb_pairs"]}


def main():
    ap = argparse.ArgumentParser()
    g = ap.add_mutually_exclusive_group(required=True)
    g.add_argument("--record", help="write a new baseline JSON")
    g.add_argument("--check", help="compare against this baseline JSON")
    ap.add_argument("--tol", type=float, default=0.05, help="allowed slowdown (fraction)")
    ap.add_argument("--only", default="", help="comma list of point names (default: all)")
    ap.add_argument("--out", default="", help="also write this run's results here")
    args = ap.parse_args()
    from bsmr import set_default_tuning, tuning_from_env

    tuning = tuning_from_env()  # BSMR_* knobs (the library reads no env): a bad knob trips it
    set_default_tuning(tuning)
    pts = points()
    if args.only:
        keep = set(args.only.split(","))
        pts = [p for p in pts if p["name"] in keep]
    base = json.load(open(args.check))["points"] if args.check else {}
    res, worst, fails = {}, 0.0, []
    for p in pts:
        t0 = time.time()
        r = time_point(p)
        r["wall_s"] = round(time.time() - t0, 1)
        line = f"{p['name']:24s} {r['ms'] * 1e3:10.2f} us {r['gflops']:10.1f} GFLOP/s"
        if p["name"] in base:
            bp = base[p["name"]]
            b = min(bp["batches_ms"]) if bp.get("batches_ms") else bp["ms"]
            slow = r["ms"] / b - 1.0
            r["vs_baseline"] = round(slow, 4)
            worst = max(worst, slow)
            line += f"   baseline {b * 1e3:10.2f} us  {slow * 100:+6.1f} %"
            if slow > args.tol:
                line += "  slower"
        print(line, flush=True)
        res[p["name"]] = dict(p, **r)
    # box factor: the median slowdown over all points. A whole box runs a few percent faster or
    # slower than the one that recorded the baseline (r05i: +1 %, mycielskian points +2..5 %); a
    # point fails when it is more than tol slower than the box factor, and the run fails when the
    # box factor itself exceeds tol (a regression of every point)
    slows = [r["vs_baseline"] for r in res.values() if "vs_baseline" in r]
    box = statistics.median(slows) if slows else 0.0
    fails = [n for n, r in res.items() if "vs_baseline" in r and r["vs_baseline"] - max(box, 0.0) > args.tol]
    if slows and box > args.tol:
        fails.append("box_factor")
    out = {"tuning": tuning, "tol": args.tol, "points": res, "box_factor": round(box, 4),
           "worst_slowdown": round(worst, 4), "failed": fails}
    if args.record:
        with open(args.record, "w") as f:
            json.dump(out, f, indent=1)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)
    if args.check:
        print(json.dumps({"guard": "FAIL" if fails else "PASS", "failed": fails,
                          "box_factor": round(box, 4), "worst_slowdown": round(worst, 4),
                          "tuning": tuning}))
        return 1 if fails else 0
    return 0


if __name__ == "__main__":
    sys.exit(main())
