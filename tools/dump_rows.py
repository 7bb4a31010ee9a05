#!/usr/bin/env python3
"""Dump a plan's reordered rows (the BSMR permutation) of a synthetic workload to .npy, for
offline layout studies on the host (tools/sweep_sim.py).

    python3 tools/dump_rows.py --workload reddit_like --scale 1.0 --out gpurun_out/rows.npy
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sddmm-gpu_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="reddit_like")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    import numpy as np

    from bsmr import Plan, synth

    M, N, rp, ci = getattr(synth, args.workload)(args.scale)
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3)
    np.save(args.out, plan.array("reorderedRows"))
    print(plan.stats()["num_reordered_rows"])


if __name__ == "__main__":
    main()
