"""GPU: the structural self-check bsmr_plan_check (the reference's check_rphm, src/BSMR.cpp:932-953
-> 444-824, run under VALIDATE before checkSddmm, src/sddmm.cu:34-38) on device plans, and the
launch layouts it extends the check to.

* every launch layout the engine picks passes: row-block (packed / unpacked / staged by runs /
  staged in pairs / original-order rows / kept fp32 tiles / 128-byte and half rows), column-major,
  dense-sampled; each also value-checked against the oracle's host SDDMM;
* the paired row-block kernel (k_sddmm_rb_pair) runs in this suite: pair_min_items lowers its
  4,096-item threshold, the plan stats show the pair launch, and XCD lists of odd length (a pair
  whose second item is padding) are among the cases;
* a corrupted plan or layout (one array element overwritten through the library's test hook)
  fails with the reference's messages on stderr; the CLI's BSMR_VALIDATE path prints them.
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

import oracle_lib as O
import bsmr
from bsmr import BF16, F16, F32, Plan, make_data, synth
from gpu_util import half_values, run_sddmm

pytestmark = pytest.mark.gpu

FREE = 288 * 1024 ** 3
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "sddmm-gpu_amd", "bin", "BSMR-sddmm")
BIN_FI = os.path.join(ROOT, "sddmm-gpu_amd", "bin", "BSMR-sddmm-faultinject")


def _poke(plan, which, index, value, K=0, dtype=F32):
    L = bsmr.lib()
    L.bsmr_debug_plan_poke.argtypes = [C.c_void_p, C.c_int, C.c_uint64, C.c_uint32, C.c_uint32,
                                       C.c_int, C.POINTER(C.c_uint32)]
    old = C.c_uint32()
    st = L.bsmr_debug_plan_poke(plan.h, which, index, value, K, dtype, C.byref(old))
    assert st == 0, L.bsmr_last_error()
    return old.value


def _rb_items(plan, K, dtype):
    L = bsmr.lib()
    L.bsmr_debug_rb_items.argtypes = [C.c_void_p, C.c_uint32, C.c_int, C.c_void_p,
                                      C.POINTER(C.c_uint64)]
    n = C.c_uint64()
    assert L.bsmr_debug_rb_items(plan.h, K, dtype, None, C.byref(n)) == 0
    buf = np.zeros(n.value, np.uint32)
    assert L.bsmr_debug_rb_items(plan.h, K, dtype, buf.ctypes.data, C.byref(n)) == 0
    return buf[4:].reshape(-1, 4)


def _values_ok(plan, M, N, rp, ci, K, dtype):
    A = make_data(M * K)
    B = make_data(N * K)
    P = run_sddmm(plan, A, B, K, len(ci), dtype=dtype)
    Ar, Br = (A, B) if dtype == F32 else (half_values(A, dtype), half_values(B, dtype))
    ref = O.sddmm_cpu(O.CSR.from_arrays(M, N, rp, ci), K, Ar, Br)
    assert np.isfinite(P).all()
    return O.check_data(ref, P)


ZIPF = lambda: synth.random_rows(517, 4000, 60, seed=2, zipf=1.1)  # noqa: E731
WIDE = lambda: synth.random_rows(1200, 30000, 180, seed=31, zipf=1.05)  # noqa: E731

# name: (pattern, K, dtype, plan kwargs)
LAYOUTS = {
    "rowblock_packed": (ZIPF, 128, F32, {}),
    "rowblock_unpacked": (ZIPF, 128, F32, {"tuning": {"out_packed": 0}}),
    "rowblock_k32": (ZIPF, 32, F32, {}),
    "rowblock_k512": (ZIPF, 512, F32, {}),
    "staged_runs": (WIDE, 128, F32, {"tuning": {"out_staged": 1}}),
    "staged_pairs": (WIDE, 128, F32, {"tuning": {"out_staged": 1, "pair_min_items": 16}}),
    # (pairs need a layout without kept MFMA tiles: no half tile demoted by default holds >= 257)
    "staged_pairs_half": (WIDE, 256, F16, {"tuning": {"out_staged": 1, "pair_min_items": 16,
                                                      "tile_min_half": 257}}),
    "orig_rows": (lambda: synth.trefethen(3000), 64, F32, {"tuning": {"orig_rows": 1}}),
    "kept_tiles_f32": (lambda: synth.block_mask(512, 16, 0.15, seed=4), 128, F32,
                       {"layout": "rowblock", "tuning": {"tile_min_f32": 0}}),
    "half_rowblock": (ZIPF, 256, BF16, {}),
    "colmajor": (ZIPF, 128, F32, {"layout": "colmajor"}),
    "colmajor_half": (ZIPF, 128, F16, {"layout": "colmajor"}),
    "dense_sampled": (lambda: synth.uniform_mask(512, 0.1, 7), 512, BF16, {}),
    # dynamic piece batches (rows of <= 512 B; waves take batches from an LDS counter): forced on
    # packed / staged / paired / half / 128- and 256-byte-row / original-order layouts, and on a
    # pattern of many single-entry pieces per item (several batches per wave)
    "batches_packed": (ZIPF, 128, F32, {"tuning": {"batches": 1}}),
    "batches_k32": (ZIPF, 32, F32, {"tuning": {"batches": 1}}),
    "batches_k64": (ZIPF, 64, F32, {"tuning": {"batches": 1}}),
    "batches_staged": (WIDE, 128, F32, {"tuning": {"out_staged": 1, "batches": 1}}),
    "batches_pairs": (WIDE, 128, F32, {"tuning": {"out_staged": 1, "pair_min_items": 16, "batches": 1}}),
    "batches_half": (WIDE, 256, F16, {"tuning": {"out_staged": 1, "tile_min_half": 257, "batches": 1}}),
    "batches_orig": (lambda: synth.trefethen(3000), 64, F32, {"tuning": {"orig_rows": 1, "batches": 1}}),
    "batches_scattered": (lambda: synth.random_rows(4000, 60000, 40, seed=12, zipf=0.6), 128, F32,
                          {"tuning": {"batches": 1}}),
}


@pytest.mark.parametrize("name", sorted(LAYOUTS))
def test_plan_and_launch_layout_pass(name, capfd):
    pat, K, dtype, kw = LAYOUTS[name]
    M, N, rp, ci = pat()
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE, **kw)
    assert _values_ok(plan, M, N, rp, ci, K, dtype) == 0
    ok, msg = plan.check(K, dtype)
    err = capfd.readouterr().err
    assert ok, (msg, err)
    assert "Error!" not in err
    st = plan.stats()
    if name.startswith("staged_pairs"):
        slot = {128: 2, 256: 2}[K]  # 512-byte rows
        assert st["rb_pairs"] & (1 << slot), st
    elif name.startswith("staged"):
        assert st["rb_pairs"] == 0
    if name == "orig_rows":
        assert st["rb_orig_rows"] != 0
    if name == "kept_tiles_f32":
        assert max(st["rb_tiles"]) > 0
    if name.startswith("batches"):
        assert st["rb_batches"] != 0, st
    if name == "batches_pairs":
        assert st["rb_pairs"] & (1 << 2), st


def test_pairs_with_padding_inside_a_pair():
    """k_sddmm_rb_pair runs list positions 2j and 2j + 1 of an XCD; a list of odd length ends in a
    pair whose second item is padding (never a padding first item: padding is a suffix). Patterns
    whose lists have odd lengths (unsplit banded row blocks dealt by the slot model, cost-cut
    chunks) must compute every entry (pairs untested)."""
    found_odd = 0
    cases = [(synth.banded_fem_like(30000, 22, 5, band=48), {}),
             (synth.banded_fem_like(21000, 18, 6, band=40), {}),
             (synth.random_rows(1200, 30000, 180, seed=33, zipf=1.05), {}),
             (synth.random_rows(1500, 40000, 150, seed=32, zipf=1.1), {}),
             (synth.random_rows(1100, 25000, 170, seed=34, zipf=1.05), {"item_cap": 1.0})]
    for (M, N, rp, ci), extra in cases:
        plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE,
                    tuning=dict({"out_staged": 1, "pair_min_items": 16}, **extra))
        assert _values_ok(plan, M, N, rp, ci, 128, F32) == 0
        assert plan.stats()["rb_pairs"] & (1 << 2)
        items = _rb_items(plan, 128, F32)
        real = (items[:, 1] > 0) | (items[:, 2] > 0)
        lists = real.reshape(-1, 8)  # [list position j, XCD x]
        for x in range(8):
            col = lists[:, x]
            n = int(col.sum())
            assert col[:n].all() and not col[n:].any(), "padding must be a suffix of each list"
            found_odd += n % 2
        ok, msg = plan.check(128, F32, verbose=False)
        assert ok, msg
    assert found_odd > 0, "no XCD list of odd length among the patterns"


def _case_plan(kw=None, K=128):
    M, N, rp, ci = synth.random_rows(600, 3000, 50, seed=9, zipf=1.2, empty_frac=0.05)
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE, **(kw or {}))
    return plan, (M, N, rp, ci)


@pytest.mark.parametrize("kind", ["rows", "dense_cols", "block_values", "sparse_values",
                                  "layout_meta", "layout_piece", "colmajor_out"])
def test_corrupted_plan_fails_with_reference_text(kind, capfd):
    kw = {"layout": "colmajor"} if kind == "colmajor_out" else None
    plan, (M, N, rp, ci) = _case_plan(kw)
    K = 128
    ok, msg = plan.check(K, F32)
    assert ok, msg
    capfd.readouterr()
    rows = plan.array("reorderedRows")
    if kind == "rows":
        _poke(plan, 0, 1, int(rows[0]))
        line, summary = "Error! Row is duplicated!", "Error! The row reordering is incorrect!"
    elif kind == "dense_cols":
        dco = plan.array("denseColOffsets")
        q = int(np.nonzero(np.diff(dco) >= 16)[0][0])
        _poke(plan, 1, int(dco[q]), N + 5)
        line, summary = "Error! Column indexes in the row panel is incorrect!", \
            "Error! The col reordering is incorrect!"
    elif kind == "block_values":
        bv = plan.array("blockValues")
        i = int(np.nonzero(bv != 0xFFFFFFFF)[0][3])
        _poke(plan, 7, i, 0xFFFFFFFF)
        line, summary = "Error! Missing value!", "Error! The rphm is incorrect!"
    elif kind == "sparse_values":
        sv = plan.array("sparseValues")
        _poke(plan, 8, 0, int(sv[1]))
        line, summary = "Error! The sparse value is incorrect!", "Error! The rphm is incorrect!"
    elif kind == "layout_meta":
        old = _poke(plan, 100, 5, 0, K, F32)  # entry 5's local row and column / position bits
        if old == 0:
            _poke(plan, 100, 5, 1 << 22, K, F32)
        line, summary = "Error! The launch layout is incorrect!", None
    elif kind == "layout_piece":
        old = _poke(plan, 101, 1, 0, K, F32)  # piece 0's column word
        _poke(plan, 101, 1, (old & ~((1 << 22) - 1)) | (((old & ((1 << 22) - 1)) + 1) % N), K, F32)
        line, summary = "Error! The launch layout is incorrect!", None
    else:
        if _poke(plan, 102, 0, 0) == 0:  # residual entry 0's output position
            _poke(plan, 102, 0, 1)
        line, summary = "Error! The launch layout is incorrect!", None
    ok, msg = plan.check(K, F32)
    err = capfd.readouterr().err
    assert not ok and line in msg and line in err, (msg, err)
    if summary:
        assert summary in err


def test_cli_validate_runs_plan_check(tmp_path):
    """BSMR_VALIDATE=1: check_rphm before checkSddmm (sddmm.cu:35-37). Clean: no error line.
    Fault-injection build with a duplicated reordered row: the reference's two lines on stderr."""
    M, N, rp, ci = synth.random_rows(500, 1500, 30, seed=13, zipf=1.05)
    path = str(tmp_path / "v.mtx")
    synth.write_mtx(path, M, N, rp, ci)
    env = dict(os.environ, BSMR_VALIDATE="1")
    r = subprocess.run([BIN, "-f", path, "-k", "64"], capture_output=True, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0, r.stderr
    assert "Error!" not in r.stderr and "NO PASS" not in r.stdout
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3)
    rows = plan.array("reorderedRows")
    env["BSMR_VALIDATE_CORRUPT_PLAN"] = f"0:1:{int(rows[0])}"
    r = subprocess.run([BIN, "-f", path, "-k", "64"], capture_output=True, text=True, timeout=300,
                       env=env)  # the release binary has no hook
    assert r.returncode == 0 and "Error!" not in r.stderr, r.stderr
    r = subprocess.run([BIN_FI, "-f", path, "-k", "64"], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    assert f"Error! Row is duplicated! Duplicated row: {int(rows[0])}" in r.stderr
    assert "Error! The row reordering is incorrect!" in r.stderr
