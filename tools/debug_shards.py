#!/usr/bin/env python3
"""Shard-launch check against the host SDDMM: the whole-plan launch and, per world size, every
shard through bsmr_sddmm_panels (global A) and bsmr_sddmm_panels_local (the shard's own A rows),
each into a NaN-filled P: unwritten entries, checkData errors, and a few wrong entries."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sddmm-gpu_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="reddit_like")
    ap.add_argument("--scale", type=float, default=0.05)
    ap.add_argument("--K", type=int, default=128)
    ap.add_argument("--worlds", default="2,4")
    args = ap.parse_args()
    import torch

    from bsmr import Plan, check_data, make_data, sddmm_cpu, set_default_tuning, synth, tuning_from_env

    gen = getattr(synth, args.workload)
    M, N, rp, ci = gen(args.scale)
    K = args.K
    set_default_tuning(tuning_from_env())
    plan = Plan(M, N, rp, ci)
    A, B = make_data(M * K), make_data(N * K)
    ref = sddmm_cpu(M, N, rp, ci, K, A, B)
    dA, dB = torch.from_numpy(A).cuda(), torch.from_numpy(B).cuda()
    nnz = len(ci)
    dP = torch.full((nnz,), float("nan"), device="cuda")
    plan.sddmm(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr())
    P = dP.cpu().numpy()
    out = {"M": M, "N": N, "nnz": nnz, "stats": {k: plan.stats()[k] for k in ("rb_rows", "rb_items")},
           "whole": {"unwritten": int(np.isnan(P).sum()), "errors": check_data(ref, P)}}
    rows = plan.array("reorderedRows")
    for world in [int(w) for w in args.worlds.split(",")]:
        res = []
        for r in range(world):
            p0, p1 = plan.shard(K, r, world)
            dP.fill_(float("nan"))
            plan.sddmm_panels(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), p0, p1)
            Pg = dP.cpu().numpy()
            # local: the shard's A rows in reordered order
            rws = np.asarray(rows, dtype=np.int64)[16 * p0:min(16 * p1, len(rows))]
            a_loc = torch.from_numpy(np.ascontiguousarray(A.reshape(M, K)[rws])).cuda()
            dP2 = torch.full((nnz,), float("nan"), device="cuda")
            plan.sddmm_panels_local(a_loc.data_ptr(), dB.data_ptr(), K, dP2.data_ptr(), p0, p1)
            Pl = dP2.cpu().numpy()
            wrote_g, wrote_l = ~np.isnan(Pg), ~np.isnan(Pl)
            bad_g = np.nonzero(wrote_g & (np.abs(Pg - ref) > 1e-3 * np.maximum(1, np.abs(ref))))[0]
            bad_l = np.nonzero(wrote_l & (np.abs(Pl - ref) > 1e-3 * np.maximum(1, np.abs(ref))))[0]
            res.append({"panels": [p0, p1], "written_global": int(wrote_g.sum()),
                        "written_local": int(wrote_l.sum()),
                        "same_written_set": bool((wrote_g == wrote_l).all()),
                        "bad_global": int(len(bad_g)), "bad_local": int(len(bad_l)),
                        "bad_local_sample": [(int(e), float(Pl[e]), float(ref[e])) for e in bad_l[:5]]})
        out[f"world{world}"] = res
    print(json.dumps(out))


if __name__ == "__main__":
    main()
