"""GPU parity of the panel-grouped tile launch (sddmm_half.hip k_sddmm_ptile): every BSMR dense
tile on `v_mfma_f32_16x16x32_{f16,bf16}`, a panel's A rows staged once per item — the reference's
tile kernel (src/sddmmKernel.cu:213-351, launched per row panel at 2570-2581) for the tile-dominated
fp16 / bf16 patterns of BASELINE.json C5 (16 x 16 block masks).

Each P is compared with the oracle's host SDDMM (src/host.cpp:45-76) on the same fp16/bf16-rounded
operands (a product of two halves is exact in fp32, so checkData's 1e-3 rule applies unchanged);
the output buffer starts as NaN, so a position no tile or residual slot writes fails the test.
"""
import numpy as np
import pytest

import oracle_lib as O
from bsmr import Plan, make_data, synth
from gpu_util import half_values, run_sddmm, torch_cuda

pytestmark = pytest.mark.gpu

FREE = 288 * 1024 ** 3


def _ref(M, N, rp, ci, K, A, B, dtype):
    return O.sddmm_cpu(O.CSR.from_arrays(M, N, rp, ci), K, half_values(A, dtype),
                       half_values(B, dtype))


def _check(plan, M, N, rp, ci, K, dtype):
    A = make_data(M * K)
    B = make_data(N * K)
    P = run_sddmm(plan, A, B, K, len(ci), dtype=dtype)
    assert np.isfinite(P).all(), f"{int((~np.isfinite(P)).sum())} outputs never written"
    ref = _ref(M, N, rp, ci, K, A, B, dtype)
    assert O.check_data(ref, P) == 0
    return P


@pytest.mark.parametrize("K", [64, 128, 256, 512])
@pytest.mark.parametrize("dtype", [1, 2])
def test_block_mask_every_tile_on_mfma(K, dtype):
    """A 16 x 16 block mask (C5's shape, smaller): the auto rule takes the panel-tile launch, every
    stored entry sits in a full BSMR tile, and the layout check passes."""
    M, N, rp, ci = synth.block_mask(512, 16, 0.15, seed=11)
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE)
    st = plan.stats()
    assert st["num_residual"] == 0 and st["num_dense_tiles"] > 0
    _check(plan, M, N, rp, ci, K, dtype)
    assert plan.stats()["ptile_items"] > 0  # the launch ran (its item list was built)
    assert plan.check(K, dtype, verbose=False) == (True, "")


@pytest.mark.parametrize("tpi", [0, 1, 3, 8, 64])
def test_tiles_per_item(tpi):
    """Items of 1..64 tiles of one panel (4 or 8 waves per workgroup, looping over the item's
    tiles past one per wave), and the default equal runs of up to two panels (tpi 0)."""
    M, N, rp, ci = synth.block_mask(768, 16, 0.2, seed=12)
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE,
                tuning={"ptile_tpi": tpi})
    _check(plan, M, N, rp, ci, 256, 2)
    assert plan.check(256, 2, verbose=False) == (True, "")


@pytest.mark.parametrize("dtype", [1, 2])
def test_forced_on_a_plan_with_residual(dtype):
    """BSMR_PTILE = 1 on a plan with partial tiles, sentinel columns and a residual (rows of M % 16,
    empty rows): tiles through the items, the residual through the column-major slots of the same
    launch (workgroups past the items)."""
    M, N, rp, ci = synth.random_rows(700, 900, 60, seed=13, zipf=1.2, empty_frac=0.05)
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE, tuning={"ptile": 1})
    st = plan.stats()
    assert st["num_dense_tiles"] > 0 and st["num_residual"] > 0
    _check(plan, M, N, rp, ci, 128, dtype)
    assert plan.stats()["ptile_items"] > 0
    assert plan.check(128, dtype, verbose=False) == (True, "")


def test_c5_block_full_size_matches_dense_sampled():
    """BASELINE.json C5 block (2048^2, 16 x 16 blocks at 10 %, bf16 K = 512): the panel-tile launch
    against the oracle, and bit for bit against the dense-sampled launch (same products, each a
    k-ordered MFMA chain of exact products in fp32 — summation order may differ, so the oracle's
    tolerance, not equality, is the parity bar; equal values are reported)."""
    M, N, rp, ci = synth.dlmc_like("block")
    K = 512
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE)
    P = _check(plan, M, N, rp, ci, K, 2)
    assert plan.stats()["ptile_items"] > 0
    dense = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE, tuning={"ptile": 0})
    P2 = _check(dense, M, N, rp, ci, K, 2)
    assert dense.stats()["dense_sampled_tiles"] > 0
    assert O.check_data(P2, P) == 0


def test_batched_launch():
    """bsmr_sddmm_batch on the panel-tile launch: grid.y = batch, reference strides."""
    torch = torch_cuda()
    M, N, rp, ci = synth.block_mask(256, 16, 0.2, seed=14)
    K, nb, nnz = 128, 3, len(ci)
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE)
    A = make_data(nb * M * K)
    B = make_data(nb * N * K)[::-1].copy()
    dA = torch.from_numpy(A).cuda().to(torch.bfloat16)
    dB = torch.from_numpy(B).cuda().to(torch.bfloat16)
    dP = torch.full((nb * nnz,), float("nan"), dtype=torch.float32, device="cuda")
    plan.sddmm_batch(nb, dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), dtype=2)
    torch.cuda.synchronize()
    P = dP.cpu().numpy()
    for b in range(nb):
        ref = _ref(M, N, rp, ci, K, A[b * M * K:(b + 1) * M * K], B[b * N * K:(b + 1) * N * K], 2)
        assert O.check_data(ref, P[b * nnz:(b + 1) * nnz]) == 0
    assert plan.stats()["ptile_items"] > 0


@pytest.mark.parametrize("word", ["row", "column", "tiles"])
def test_corrupted_descriptor_fails_the_layout_check(word):
    """bsmr_plan_check verifies the descriptors the panel-tile kernel reads (rows, tile range,
    columns) against the plan; one corrupted word fails with the descriptor's message."""
    from test_gpu_plan_check import _poke
    M, N, rp, ci = synth.block_mask(512, 16, 0.15, seed=15)
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE)
    assert plan.check(256, 2, verbose=False) == (True, "")  # builds the descriptors
    items = plan.stats()["ptile_items"]
    assert items > 0
    # the first item slot with tiles (slot 0 holds the XCD-0 eighth's first item)
    idx = {"row": 3, "column": 48 + 5, "tiles": 33}[word]
    old = _poke(plan, 103, idx, 7, 256, 2)
    _poke(plan, 103, idx, old ^ 1 if word != "tiles" else old + 1, 256, 2)
    ok, msg = plan.check(256, 2, verbose=False)
    assert not ok and "panel-tile descriptor" in msg, msg


@pytest.mark.parametrize("scale", [1, 3])
def test_equal_runs_across_panel_boundaries(scale):
    """The default item list (equal tile runs, one per CU): with more tiles than CUs most runs
    cross a panel boundary and stage both panels' A rows (32 rows in LDS, the second panel's
    tiles reading rows 16..31); with 3x the tiles of C5 a run holds up to 8 tiles (more runs than
    CUs). Every output equals the oracle's, and the layout check covers both panels' rows."""
    M, N, rp, ci = synth.block_mask(1024 * scale, 16, 0.1, seed=16)
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE)
    st = plan.stats()
    assert st["num_residual"] == 0 and st["num_dense_tiles"] > 256
    _check(plan, M, N, rp, ci, 512, 2)
    assert plan.check(512, 2, verbose=False) == (True, "")
