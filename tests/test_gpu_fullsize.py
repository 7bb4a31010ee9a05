"""GPU parity at BASELINE.json's full workload sizes (not samples): every stored entry of the
HIP SDDMM against the oracle's host SDDMM (host.cpp:45-76 loop order) by the checkData rule
(|a-b| < 1e-5 or |a-b| / max(|a|, |b|, 1e-3) < 1e-3, checkData.hpp:14-30), zero mismatches.

* C2 nips-like, fp32, K = 128 (the bench line's workload);
* C3 cop20k_A-like 121,192^2, fp16 A/B (the oracle runs in fp32 on the same rounded values:
  half x half products are exact in fp32), K = 256;
* C4 reddit-like at its BASELINE size (232,965^2, 232 M stored entries), fp32, K = 128, in the
  three forms bench.py runs: the whole-plan launch, the 8-way row-panel split of the one global
  plan (bsmr_sddmm_panels_local, shard-local A rows) and the 8 local per-panel plans (contiguous
  original row panels of equal stored entries, each with its own plan);
* C5 DLMC-like 2048^2 90 %-sparse masks (uniform: the dense-sampled MFMA launch; 16x16 blocks: the
  column-major tile launch), bf16, K = 512.
Each plan also passes bsmr_plan_check (check_rphm + its launch layout) at that size.
"""
import functools

import numpy as np
import pytest

import oracle_lib as O
from bsmr import BF16, F16, F32, Plan, make_data, synth
from bsmr import dist as D
from gpu_util import half_values, torch_cuda

pytestmark = pytest.mark.gpu


@functools.lru_cache(maxsize=None)
def _pattern(name):
    if name == "C2":
        return synth.nips_like()
    if name == "C3":
        return synth.cop20k_like()
    if name == "C4":
        return synth.reddit_like(1.0)
    return synth.dlmc_like(name[3:])


def _gpu(plan, A, B, K, nnz, dtype, shards=None, rows=None):
    torch = torch_cuda()
    tdt = {F32: torch.float32, F16: torch.float16, BF16: torch.bfloat16}[dtype]
    dB = torch.from_numpy(B).cuda().to(tdt)
    dP = torch.full((nnz,), float("nan"), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    if shards is None:
        dA = torch.from_numpy(A).cuda().to(tdt)
        plan.sddmm(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), stream=s, dtype=dtype)
        torch.cuda.synchronize()
    else:
        for p0, p1 in shards:
            dA = torch.from_numpy(D.shard_a_rows(A, K, rows, p0, p1).reshape(-1)).cuda().to(tdt)
            plan.sddmm_panels_local(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), p0, p1,
                                    stream=s, dtype=dtype)
            torch.cuda.synchronize()
            del dA
    return dP.cpu().numpy()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("name,K,dtype", [("C2", 128, F32), ("C3", 256, F16), ("C4", 128, F32),
                                          ("C5_uniform", 512, BF16), ("C5_block", 512, BF16)])
def test_full_workload_every_entry(name, K, dtype):
    M, N, rp, ci = _pattern(name)
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3)
    A = make_data(M * K)
    B = make_data(N * K)
    Ar, Br = (A, B) if dtype == F32 else (half_values(A, dtype), half_values(B, dtype))
    ref = O.sddmm_cpu(O.CSR.from_arrays(M, N, rp, ci), K, Ar, Br)
    P = _gpu(plan, A, B, K, len(ci), dtype)
    assert np.isfinite(P).all()
    assert O.check_data(ref, P) == 0
    del P
    # the reference's structural self-check (check_rphm, BSMR.cpp:932-953) and the launch layout
    # of (K, dtype): every stored entry computed exactly once, at the full size
    ok, msg = plan.check(K, dtype)
    assert ok, msg
    if name == "C4":  # the north_star split: 8 row-panel shards, each with only its A rows
        rows = plan.array("reorderedRows")
        shards = [plan.shard(K, r, 8, dtype) for r in range(8)]
        assert shards[0][0] == 0 and shards[-1][1] == plan.stats()["num_row_panels"]
        assert all(a[1] == b[0] for a, b in zip(shards, shards[1:]))
        Ps = _gpu(plan, A, B, K, len(ci), dtype, shards=shards, rows=rows)
        assert np.isfinite(Ps).all()
        assert O.check_data(ref, Ps) == 0
        del Ps, plan
        # the local split: 8 contiguous original row panels, each planned on its own
        torch = torch_cuda()
        dB = torch.from_numpy(B).cuda()
        dP = torch.full((len(ci),), float("nan"), dtype=torch.float32, device="cuda")
        rp64 = np.asarray(rp, dtype=np.int64)
        for r in range(8):
            r0, r1 = D.row_range_cut(rp64, r, 8)
            e0, e1 = int(rp64[r0]), int(rp64[r1])
            lp = Plan(r1 - r0, N, (rp64[r0:r1 + 1] - e0).astype(np.uint32), ci[e0:e1],
                      alpha=0.3, delta=0.3)
            dA = torch.from_numpy(np.ascontiguousarray(A[r0 * K:r1 * K])).cuda()
            lp.sddmm(dA.data_ptr(), dB.data_ptr(), K, dP[e0:e1].data_ptr(),
                     stream=torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            del lp, dA
        Pl = dP.cpu().numpy()
        assert np.isfinite(Pl).all()
        assert O.check_data(ref, Pl) == 0
