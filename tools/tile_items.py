#!/usr/bin/env python3
"""Per-item kept-tile / entry / piece counts of a row-block layout (bsmr_debug_rb_items) under the
current BSMR_* tuning, e.g. BSMR_TILE_MIN_F32=0 python3 tools/tile_items.py --workload nips_like"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sddmm-gpu_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="nips_like")
    ap.add_argument("--K", type=int, default=128)
    ap.add_argument("--dtype", type=int, default=0)
    args = ap.parse_args()
    import bsmr
    from bsmr import Plan, make_data, set_default_tuning, synth, tuning_from_env
    import torch

    set_default_tuning(tuning_from_env())
    M, N, rp, ci = getattr(synth, args.workload)()
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3)
    K = args.K
    tdt = {0: torch.float32, 1: torch.float16, 2: torch.bfloat16}[args.dtype]
    dA = torch.from_numpy(make_data(M * K)).cuda().to(tdt)
    dB = torch.from_numpy(make_data(N * K)).cuda().to(tdt)
    dP = torch.zeros(len(ci), dtype=torch.float32, device="cuda")
    plan.sddmm(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), dtype=args.dtype)
    torch.cuda.synchronize()
    L = bsmr.lib()
    L.bsmr_debug_rb_items.argtypes = [C.c_void_p, C.c_uint32, C.c_int, C.c_void_p, C.POINTER(C.c_uint64)]
    n = C.c_uint64()
    L.bsmr_debug_rb_items(plan.h, K, args.dtype, None, C.byref(n))
    buf = np.zeros(n.value, np.uint32)
    L.bsmr_debug_rb_items(plan.h, K, args.dtype, buf.ctypes.data, C.byref(n))
    hdr, it = buf[:4], buf[4:].reshape(-1, 4)
    real = (it[:, 1] > 0) | (it[:, 2] > 0)
    it = it[real]
    pct = lambda x: [int(v) for v in np.percentile(x, [0, 10, 50, 90, 100])]  # noqa: E731
    print(json.dumps({"RB": int(hdr[0]), "NT": int(hdr[1]), "items": int(real.sum()),
                      "tiles": pct(it[:, 1]), "entries": pct(it[:, 2]), "pieces": pct(it[:, 3]),
                      "items_over_16_tiles": int((it[:, 1] > 16).sum()),
                      "tiles_total": int(it[:, 1].sum()), "entries_total": int(it[:, 2].sum()),
                      "pieces_total": int(it[:, 3].sum())}))


if __name__ == "__main__":
    main()
