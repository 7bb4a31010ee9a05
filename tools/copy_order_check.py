#!/usr/bin/env python3
"""One C2-sized copy of bench.py's weak-scaling stack on its own plan (through gpurun): copy 0
(the nips-like pattern), copy 1 (columns relabelled; synth.stack_copies keeps every row's columns
ascending) and copy 1 with each row's columns shuffled (CSR order = an unsorted file's order);
prints the SDDMM ms of each (bsmr_sddmm_profile)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sddmm-gpu_amd"))
from bsmr import Plan, make_data, synth  # noqa: E402

M, N, rp, ci = synth.nips_like()
K = 128
Ms, _, rps, cis = synth.stack_copies(M, N, rp, ci, 2)
rps = np.asarray(rps, np.int64)
b0, b1 = int(rps[M]), int(rps[2 * M])
rp1 = (rps[M:2 * M + 1] - b0).astype(np.uint32)
ci1 = np.asarray(cis[b0:b1], np.uint32)
ci1u = ci1.copy()
rng = np.random.default_rng(5)
for r in range(M):
    rng.shuffle(ci1u[rp1[r]:rp1[r + 1]])
dA = torch.from_numpy(make_data(M * K)).cuda()
dB = torch.from_numpy(make_data(N * K)).cuda()
out = {}
for name, (r_, c_) in {"copy0": (rp, ci), "copy1_sorted": (rp1, ci1),
                       "copy1_unsorted": (rp1, ci1u)}.items():
    p = Plan(M, N, np.asarray(r_, np.uint32), np.asarray(c_, np.uint32), alpha=0.3, delta=0.3)
    dP = torch.zeros(len(c_), dtype=torch.float32, device="cuda")
    out[name] = p.profile(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), iters=50)
    out[name + "_stats"] = {k: v for k, v in p.stats().items() if "rb_" in k or "cluster" in k}
print(json.dumps(out))
