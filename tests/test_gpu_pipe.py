"""GPU: the pipelined row-block launch (k_sddmm_rb_pipe, bsmr_tuning.pipe): one
persistent workgroup per CU takes its XCD bucket's list items from a counter, two waves stage the
next item's A rows into a second LDS image while fourteen run the current item's pieces.

* every entry is computed (checkData against the oracle's host SDDMM) on staged-output patterns of
  512-byte rows: fp32 K = 128, fp16 / bf16 K = 256, original-order banded rows, one item per
  segment (lists of odd length, padding items), and the plan stats show the pipelined launch;
* repeated launches give bit-identical P (the per-XCD counters are reset by each launch's last
  workgroup), also interleaved with launches of another pipelined plan on the same stream;
* the layout passes bsmr_plan_check, and a batched launch of a pipelined layout (which runs its
  items on k_sddmm_rb) computes every batch.
"""
import numpy as np
import pytest

import oracle_lib as O
from bsmr import BF16, F16, F32, Plan, make_data, synth
from gpu_util import half_values, run_sddmm, torch_cuda

pytestmark = pytest.mark.gpu

FREE = 288 * 1024 ** 3
SLOT512 = 2  # stats index of the 512-byte-row layout

CASES = {
    "wide_f32": (lambda: synth.random_rows(1200, 30000, 180, seed=31, zipf=1.05), 128, F32, {}),
    "wide_f16": (lambda: synth.random_rows(1200, 30000, 180, seed=31, zipf=1.05), 256, F16,
                 {"tile_min_half": 257}),
    "wide_bf16_odd_lists": (lambda: synth.random_rows(1500, 40000, 150, seed=32, zipf=1.1), 256, BF16,
                            {"tile_min_half": 257, "seg_items": 1}),
    "banded_orig_f16": (lambda: synth.banded_fem_like(30000, 22, 5, band=48), 256, F16,
                        {"orig_rows": 1}),
    "zipf_f32_seg1": (lambda: synth.random_rows(2000, 20000, 120, seed=7, zipf=1.2), 128, F32,
                      {"seg_items": 1}),
}


def _plan(name, pipe=1):
    pat, K, dtype, extra = CASES[name]
    M, N, rp, ci = pat()
    tuning = dict({"out_staged": 1, "pipe": pipe}, **extra)
    return (M, N, rp, ci, K, dtype), Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE,
                                          tuning=tuning)


def _ref(M, N, rp, ci, K, dtype, A, B):
    Ar, Br = (A, B) if dtype == F32 else (half_values(A, dtype), half_values(B, dtype))
    return O.sddmm_cpu(O.CSR.from_arrays(M, N, rp, ci), K, Ar, Br)


@pytest.mark.parametrize("name", sorted(CASES))
def test_pipe_values_and_check(name):
    (M, N, rp, ci, K, dtype), plan = _plan(name)
    A, B = make_data(M * K), make_data(N * K)
    P = run_sddmm(plan, A, B, K, len(ci), dtype=dtype)
    assert np.isfinite(P).all(), "an entry was not written"
    assert O.check_data(_ref(M, N, rp, ci, K, dtype, A, B), P) == 0
    st = plan.stats()
    assert st["rb_pipe"] & (1 << SLOT512), st
    assert st["rb_pairs"] == 0 and st["rb_sweep"] == 0
    ok, msg = plan.check(K, dtype, verbose=False)
    assert ok, msg


def test_pipe_repeated_launches_bit_identical():
    torch = torch_cuda()
    (M, N, rp, ci, K, dtype), plan = _plan("wide_f32")
    (M2, N2, rp2, ci2, K2, dt2), plan2 = _plan("zipf_f32_seg1")
    s = torch.cuda.current_stream().cuda_stream
    dA = torch.from_numpy(make_data(M * K)).cuda()
    dB = torch.from_numpy(make_data(N * K)).cuda()
    dA2 = torch.from_numpy(make_data(M2 * K2)).cuda()
    dB2 = torch.from_numpy(make_data(N2 * K2)).cuda()
    outs, outs2 = [], []
    for _ in range(4):
        dP = torch.full((len(ci),), float("nan"), dtype=torch.float32, device="cuda")
        dP2 = torch.full((len(ci2),), float("nan"), dtype=torch.float32, device="cuda")
        plan.sddmm(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), stream=s, dtype=dtype)
        plan2.sddmm(dA2.data_ptr(), dB2.data_ptr(), K2, dP2.data_ptr(), stream=s, dtype=dt2)
        torch.cuda.synchronize()
        outs.append(dP.cpu().numpy())
        outs2.append(dP2.cpu().numpy())
    for o in outs[1:]:
        assert np.array_equal(o, outs[0])
    for o in outs2[1:]:
        assert np.array_equal(o, outs2[0])
    assert np.isfinite(outs[0]).all() and np.isfinite(outs2[0]).all()


def test_pipe_matches_unpipelined_layout():
    (M, N, rp, ci, K, dtype), plan = _plan("wide_f16")
    _, plain = _plan("wide_f16", pipe=0)
    A, B = make_data(M * K), make_data(N * K)
    P = run_sddmm(plan, A, B, K, len(ci), dtype=dtype)
    Q = run_sddmm(plain, A, B, K, len(ci), dtype=dtype)
    assert plain.stats()["rb_pipe"] == 0
    # the same entries in both layouts; summation order per entry may differ (row-group rotation)
    assert O.check_data(Q, P) == 0


def test_pipe_layout_batched_launch():
    torch = torch_cuda()
    (M, N, rp, ci, K, dtype), plan = _plan("wide_f32")
    nb = 3
    A = [make_data(M * K) * (b + 1) for b in range(nb)]
    B = [make_data(N * K) for _ in range(nb)]
    dA = torch.from_numpy(np.concatenate(A)).cuda()
    dB = torch.from_numpy(np.concatenate(B)).cuda()
    dP = torch.full((nb * len(ci),), float("nan"), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    plan.sddmm_batch(nb, dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), stream=s, dtype=dtype)
    torch.cuda.synchronize()
    P = dP.cpu().numpy().reshape(nb, -1)
    for b in range(nb):
        assert O.check_data(_ref(M, N, rp, ci, K, dtype, A[b], B[b]), P[b]) == 0
