"""GPU parity of the column-block launch (round 6): on wide patterns the row-block kernel runs with
the operands' roles swapped — blocks of ORIGINAL columns, their B rows staged in LDS, each piece a
run of one A row over the block's columns (plan.hip `build_rowblock_layout(.., cols)`,
sddmm.hip `launch_rb`). The plan's RPHM arrays are untouched (the reference's BSMR plan,
src/BSMR.cpp); only the launch order of the same dot products changes, so every P is held to the
oracle's host SDDMM (src/host.cpp:45-76) by the reference's checkData rule, and the output buffer
starts as NaN so a position no piece writes fails the test.
"""
import numpy as np
import pytest

import oracle_lib as O
from bsmr import BF16, F16, F32, Plan, make_data, synth
from gpu_util import half_values, run_sddmm, torch_cuda

pytestmark = pytest.mark.gpu

FREE = 288 * 1024 ** 3
SLOT = {32: 0, 64: 1, 128: 2, 256: 3, 512: 4}  # fp32 row size -> stats bit


def _check(plan, M, N, rp, ci, K, dtype=F32):
    A = make_data(M * K)
    B = make_data(N * K)[::-1].copy()
    P = run_sddmm(plan, A, B, K, len(ci), dtype=dtype)
    assert np.isfinite(P).all(), f"{int((~np.isfinite(P)).sum())} outputs never written"
    Ar, Br = (A, B) if dtype == F32 else (half_values(A, dtype), half_values(B, dtype))
    ref = O.sddmm_cpu(O.CSR.from_arrays(M, N, rp, ci), K, Ar, Br)
    assert O.check_data(ref, P) == 0
    return P


def test_c2_piece_rule_takes_column_blocks():
    """BASELINE.json C2 (nips-like 1,500 x 12,419, fp32 K = 128): the piece rule (col_blocks = 2)
    picks column blocks (N >= 2 M, pieces below 0.9 x the row-block layout's), P matches the
    oracle and the layout check passes entry by entry; the default keeps row blocks."""
    M, N, rp, ci = synth.nips_like()
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE, tuning={"col_blocks": 2})
    _check(plan, M, N, rp, ci, 128)
    st = plan.stats()
    assert st["rb_col_blocks"] & (1 << SLOT[128]), st
    assert plan.check(128, F32, verbose=False) == (True, "")
    off = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE)
    _check(off, M, N, rp, ci, 128)
    assert off.stats()["rb_col_blocks"] == 0
    assert st["rb_pieces"][SLOT[128]] < 0.9 * off.stats()["rb_pieces"][SLOT[128]]


@pytest.mark.parametrize("K", [32, 64, 128, 256, 512])
@pytest.mark.parametrize("shape", ["wide", "square", "tall"])
def test_forced_column_blocks_fp32(K, shape):
    """BSMR_COL_BLOCKS = 1 on wide, square and tall patterns with empty rows and a Zipf column
    law, every fp32 row size (128 B .. 2 KiB)."""
    M, N = {"wide": (600, 5000), "square": (1500, 1500), "tall": (4000, 500)}[shape]
    M, N, rp, ci = synth.random_rows(M, N, 30, seed=21 + K, zipf=1.1, empty_frac=0.05)
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE, tuning={"col_blocks": 1})
    _check(plan, M, N, rp, ci, K)
    assert plan.stats()["rb_col_blocks"] & (1 << SLOT[K])
    assert plan.check(K, F32, verbose=False) == (True, "")


@pytest.mark.parametrize("dtype", [F16, BF16])
@pytest.mark.parametrize("K", [64, 256])
def test_forced_column_blocks_half(dtype, K):
    """fp16 / bf16 operands (the swizzled half image) on the column-block launch."""
    M, N, rp, ci = synth.random_rows(500, 4000, 24, seed=31, zipf=1.2)
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE, tuning={"col_blocks": 1})
    _check(plan, M, N, rp, ci, K, dtype)
    assert plan.stats()["rb_col_blocks"]
    assert plan.check(K, dtype, verbose=False) == (True, "")


@pytest.mark.parametrize("knobs", [{"out_staged": 1}, {"out_staged": 1, "pair_min_items": 0},
                                   {"batches": 1}, {"out_packed": 0}])
def test_column_blocks_output_paths(knobs):
    """The column-block layout through the staged output (LDS slots, run table), the paired kernel,
    dynamic piece batches and unpacked output positions."""
    M, N, rp, ci = synth.random_rows(800, 6000, 40, seed=41, zipf=1.1, empty_frac=0.02)
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE,
                tuning=dict(knobs, col_blocks=1))
    _check(plan, M, N, rp, ci, 128)
    assert plan.stats()["rb_col_blocks"]
    assert plan.check(128, F32, verbose=False) == (True, "")


def test_column_blocks_batched():
    """bsmr_sddmm_batch on the column-block launch: the staged operand is B, so the batch strides
    swap with the pointers."""
    torch = torch_cuda()
    M, N, rp, ci = synth.random_rows(300, 2400, 20, seed=51, zipf=1.1)
    K, nb, nnz = 128, 3, len(ci)
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE, tuning={"col_blocks": 1})
    A = make_data(nb * M * K)
    B = make_data(nb * N * K)[::-1].copy()
    dA = torch.from_numpy(A).cuda()
    dB = torch.from_numpy(B).cuda()
    dP = torch.full((nb * nnz,), float("nan"), dtype=torch.float32, device="cuda")
    plan.sddmm_batch(nb, dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr())
    torch.cuda.synchronize()
    P = dP.cpu().numpy()
    c = O.CSR.from_arrays(M, N, rp, ci)
    for b in range(nb):
        ref = O.sddmm_cpu(c, K, A[b * M * K:(b + 1) * M * K], B[b * N * K:(b + 1) * N * K])
        assert O.check_data(ref, P[b * nnz:(b + 1) * nnz]) == 0
    assert plan.stats()["rb_col_blocks"]


def test_panel_shards_of_a_column_block_plan():
    """A plan whose whole launch takes column blocks still runs its row-panel shards on the
    reordered row-block layouts (bsmr_sddmm_panels), cut by the reordered layout's costs."""
    M, N, rp, ci = synth.random_rows(900, 7000, 30, seed=61, zipf=1.1)
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE, tuning={"col_blocks": 1})
    K = 128
    A = make_data(M * K)
    B = make_data(N * K)
    whole = run_sddmm(plan, A, B, K, len(ci))
    assert plan.stats()["rb_col_blocks"]
    cuts = [plan.shard(K, r, 3) for r in range(3)]
    assert cuts[0][0] == 0 and cuts[-1][1] == plan.stats()["num_row_panels"]
    P = run_sddmm(plan, A, B, K, len(ci), panels=cuts)
    assert np.isfinite(P).all()
    ref = O.sddmm_cpu(O.CSR.from_arrays(M, N, rp, ci), K, A, B)
    assert O.check_data(ref, P) == 0 and O.check_data(ref, whole) == 0


def test_corrupted_column_block_entry_fails_the_check():
    """bsmr_plan_check verifies the column-block layout entry by entry with (row, column) swapped
    back: one corrupted metadata word fails it."""
    from test_gpu_plan_check import _poke
    M, N, rp, ci = synth.random_rows(400, 3000, 20, seed=71, zipf=1.1)
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE, tuning={"col_blocks": 1})
    assert plan.check(128, F32, verbose=False) == (True, "")
    old = _poke(plan, 100, 5, 0, 128, F32)
    _poke(plan, 100, 5, old ^ 1, 128, F32)
    ok, msg = plan.check(128, F32, verbose=False)
    assert not ok and "item" in msg, msg
