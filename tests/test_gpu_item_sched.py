"""Row-block item scheduling on the reference's own matrices: the values
are the host SDDMM's under every scheduling switch, no item exceeds the cost cap, and the
small-sparse-row rule gives Trefethen one row block per workgroup slot.

Item stats come from the debug export bsmr_debug_rb_items (4 u32 per item slot: row block, kept
tiles, entries, pieces; header: rows per block, threads, items, row bytes)."""
import ctypes as C
import functools

import numpy as np
import pytest

import bsmr
import oracle_lib as O
from bsmr import Plan, make_data, synth, tuning_from_env
from gpu_util import run_sddmm

pytestmark = pytest.mark.gpu


@functools.lru_cache(maxsize=None)
def case(name):
    return synth.SUITESPARSE_REBUILDS[name]()


def rb_items(plan, K, dtype=0):
    L = bsmr.lib()
    L.bsmr_debug_rb_items.argtypes = [C.c_void_p, C.c_uint32, C.c_int, C.c_void_p,
                                      C.POINTER(C.c_uint64)]
    n = C.c_uint64()
    assert L.bsmr_debug_rb_items(plan.h, K, dtype, None, C.byref(n)) == 0
    buf = np.zeros(n.value, np.uint32)
    assert L.bsmr_debug_rb_items(plan.h, K, dtype, buf.ctypes.data, C.byref(n)) == 0
    RB, NT, nitems, row_bytes = (int(v) for v in buf[:4])
    st = buf[4:].reshape(-1, 4).astype(np.int64)
    assert len(st) == nitems
    return RB, NT, row_bytes, st


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name,K,alpha,delta", [("mycielskian14", 128, 0.3, 0.3),
                                                ("mycielskian14", 512, 0.5, 0.7),
                                                ("Trefethen_20000", 64, 0.1, 0.5)])
@pytest.mark.parametrize("env", [{}, {"BSMR_ITEM_SCHED": "0", "BSMR_ITEM_CAP": "0"},
                                 {"BSMR_ITEM_CAP": "1"}])
def test_values_under_item_scheduling(name, K, alpha, delta, env):
    M, N, rp, ci = case(name)
    plan = Plan(M, N, rp, ci, alpha=alpha, delta=delta, layout="rowblock",
                tuning=tuning_from_env(env))
    A, B = make_data(M * K), make_data(N * K)
    P = run_sddmm(plan, A, B, K, len(ci))
    ref = O.sddmm_cpu(O.CSR.from_arrays(M, N, rp, ci), K, A, B)
    assert np.isfinite(P).all()
    assert O.check_data(ref, P) == 0
    RB, NT, row_bytes, st = rb_items(plan, K)
    assert st[:, 2].sum() == len(ci)  # every stored entry in exactly one item
    assert RB % 16 == 0 and RB * row_bytes <= 160 * 1024


@pytest.mark.parametrize("name,K,alpha,delta", [("mycielskian14", 128, 0.3, 0.3),
                                                ("mycielskian15", 256, 0.5, 0.7)])
def test_no_item_above_the_cap(name, K, alpha, delta):
    """Cost cap: with item_cap = c, no item's modeled cost (entries + 4 per piece + 16 per tile)
    exceeds c x one slot's share of the launch (the staged-output split only shrinks items);
    the hub-row chunk of 8 K single-entry pieces that set round 2's mycielskian launch is gone."""
    M, N, rp, ci = case(name)
    for cap in (1.0, 2.0):
        plan = Plan(M, N, rp, ci, alpha=alpha, delta=delta, layout="rowblock",
                    tuning={"item_cap": cap})
        RB, NT, row_bytes, st = rb_items(plan, K)
        cost = st[:, 2] + 4.0 * st[:, 3] + 16.0 * st[:, 1]
        slots = 256 * (2 if NT == 512 else 1)
        share = cost.sum() / slots
        # (the cuts fall on entries, so one entry plus one piece of slack)
        assert cost.max() <= cap * share * 1.02 + 5, (cap, cost.max(), share)


def test_trefethen_one_block_per_slot():
    """Sparse-row patterns with fewer row blocks than slots: blocks of ceil(R / 512) rows rounded
    to 16 (two 80 KiB workgroups per CU), all in one round of the 512 slots (the heavier blocks
    take the slots left over; round 2: 35 blocks of 576 rows cut into 257 items that each
    restaged the whole image)."""
    M, N, rp, ci = case("Trefethen_20000")
    plan = Plan(M, N, rp, ci, alpha=0.1, delta=0.5, layout="rowblock")
    RB, NT, row_bytes, st = rb_items(plan, 64)
    assert RB == 48 and NT == 512
    work = st[:, 2] > 0
    assert work.sum() <= 512
    assert len(np.unique(st[work, 0])) == (M + RB - 1) // RB  # 417 blocks, each >= 1 item
    assert np.bincount(st[work, 0]).max() <= 2
    old = Plan(M, N, rp, ci, alpha=0.1, delta=0.5, layout="rowblock",
               tuning={"item_sched": 0, "item_cap": 0})
    assert rb_items(old, 64)[0] == 576
