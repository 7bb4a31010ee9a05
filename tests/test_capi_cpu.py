"""CPU-side checks of the C ABI library (no device calls): symbol exports, host loader and makeData
parity with the oracle and the reference's known answers."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle_lib as O
import bsmr
from bsmr import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_symbol():
    header = open(os.path.join(ROOT, "include", "bsmr.h")).read()
    declared = set(re.findall(r"\b(bsmr_[a-z_0-9]+)\s*\(", header))
    declared -= {"bsmr_plan_options", "bsmr_plan_stats", "bsmr_eval_stats"}
    L = bsmr.lib()
    missing = [s for s in sorted(declared) if not hasattr(L, s)]
    assert not missing, missing
    assert declared == set(bsmr.EXPORTS), declared ^ set(bsmr.EXPORTS)
    assert L.bsmr_abi_version() == bsmr.ABI_VERSION == 13


def test_rocsparse_baseline_exports_every_header_symbol():
    from bsmr import vendor

    header = open(os.path.join(ROOT, "include", "bsmr_rocsparse.h")).read()
    declared = set(re.findall(r"\b(bsmr_rocsparse_[a-z_0-9]+)\s*\(", header))
    L = vendor.lib()
    missing = [s for s in sorted(declared) if not hasattr(L, s)]
    assert not missing, missing
    assert declared == set(vendor.EXPORTS), declared ^ set(vendor.EXPORTS)


def test_plan_options_defaults_and_struct_size():
    """bsmr_plan_options_default fills exactly the ctypes mirror of the C struct."""
    n = ctypes.sizeof(bsmr.PlanOptions)
    buf = (ctypes.c_uint8 * (n + 32))(*([0xAB] * (n + 32)))
    bsmr.lib().bsmr_plan_options_default(ctypes.cast(buf, ctypes.POINTER(bsmr.PlanOptions)))
    assert bytes(buf[n:]) == b"\xab" * 32
    o = bsmr.PlanOptions.from_buffer(buf)
    assert abs(o.alpha - 0.3) < 1e-7 and abs(o.delta - 0.3) < 1e-7
    assert (o.free_mem_bytes, o.device, o.cluster_batch, o.exact_similarity) == (0, 0, 0, 0)
    assert (o.layout, o.lds_budget_kb) == (bsmr.LAYOUTS["auto"], 0)


def test_make_data_known_answer():
    # reference makeData stream: A[0] = B[0] = 1.62944734 (single-threaded)
    v = bsmr.make_data(4096)
    assert abs(float(v[0]) - 1.62944734) < 1e-7
    assert v.dtype == np.float32 and (v >= 0).all() and (v < 2).all()
    assert np.array_equal(v, O.make_data(4096))


MTX_CASES = {
    "ok_general": ("%%MatrixMarket matrix coordinate real general\n% c\n3 4 4\n1 1 1.0\n3 4 2\n"
                   "2 2 3\n1 3 4\n", True),
    "ok_pattern_no_values": ("%%MatrixMarket matrix coordinate pattern symmetric\n3 3 3\n2 1\n"
                             "3 1\n3 2\n", True),
    "ok_blank_lines_crlf": ("%%MM\n2 2 2\r\n1 1 5\r\n\n2 2 7\r\n", True),
    "ok_tabs": ("%x\n2 3 3\n1\t3\t1\n2\t1\t1\n1\t1\t1\n", True),
    "too_many": ("%x\n2 2 2\n1 1 1\n2 2 1\n1 2 1\n", False),
    "too_few": ("%x\n2 2 3\n1 1 1\n2 2 1\n", False),
    "out_of_range": ("%x\n2 2 2\n1 1 1\n3 2 1\n", False),
    "zero_index": ("%x\n2 2 2\n0 1 1\n2 2 1\n", False),
    "duplicate": ("%x\n2 2 3\n1 1 1\n2 2 1\n1 1 5\n", False),
    "nnz_one": ("%x\n2 2 1\n1 1 1\n", False),
    "bad_token": ("%x\n2 2 2\n1 a 1\n2 2 1\n", False),
}


@pytest.mark.parametrize("case", sorted(MTX_CASES))
def test_loader_matches_oracle(tmp_path, case):
    text, ok = MTX_CASES[case]
    path = str(tmp_path / f"{case}.mtx")
    with open(path, "w", newline="") as f:
        f.write(text)
    a = bsmr.load_mtx(path)
    o = O.CSR.load(path)
    assert (a is not None) == ok
    assert (o is not None) == ok
    if ok:
        rp, ci, v = o.arrays()
        assert (a.M, a.N, a.nnz) == (o.M, o.N, o.nnz)
        assert np.array_equal(a.rowptr, rp)
        assert np.array_equal(a.colidx, ci)
        assert np.array_equal(a.values, v)


def test_loader_keeps_file_order_within_rows(tmp_path):
    path = str(tmp_path / "order.mtx")
    with open(path, "w") as f:
        f.write("%x\n2 5 5\n2 5 1\n1 4 1\n2 1 1\n1 2 1\n2 3 1\n")
    a = bsmr.load_mtx(path)
    assert list(a.rowptr) == [0, 2, 5]
    assert list(a.colidx) == [3, 1, 4, 0, 2]


def test_wrong_suffix_rejected(tmp_path):
    path = str(tmp_path / "x.txt2")
    open(path, "w").write("%x\n2 2 2\n1 1 1\n2 2 1\n")
    assert bsmr.load_mtx(path) is None


def test_loader_roundtrip_synthetic(tmp_path):
    M, N, rp, ci = synth.random_rows(123, 777, 9, seed=5)
    path = str(tmp_path / "syn.mtx")
    synth.write_mtx(path, M, N, rp, ci)
    a = bsmr.load_mtx(path)
    assert np.array_equal(a.rowptr, rp) and np.array_equal(a.colidx, ci)


def test_shard_cuts_host_model():
    bo = np.array([0, 3, 3, 10, 12, 12], np.uint32)
    so = np.array([0, 100, 900, 950, 1000, 4000], np.uint32)
    for world in (1, 2, 3, 5, 8):
        cuts = bsmr.shard_cuts(bo, so, 128, world)
        assert cuts[0] == 0 and cuts[-1] == len(bo) - 1
        assert (np.diff(cuts.astype(np.int64)) >= 0).all()


def test_missing_library_fails_loudly(monkeypatch):
    monkeypatch.setattr(bsmr, "_lib", None)
    monkeypatch.setattr(bsmr, "LIB_PATH", "/nonexistent/libbsmr_amd.so")
    with pytest.raises(bsmr.BsmrError):
        bsmr.lib()


def test_tuning_env_parser_matches_python_mapping(monkeypatch):
    """bsmr_tuning_from_env (the library's parser, called explicitly by tools) and the Python
    mapping the tests use give the same knobs; nothing is read unless asked."""
    import bsmr
    env = {"BSMR_TILE_MIN_F32": "0", "BSMR_OUT_STAGED": "1", "BSMR_ORIG_ROWS": "auto",
           "BSMR_PIECE_WEIGHT": "2.5", "BSMR_L2_RANGE_KB": "64", "BSMR_DIAG": "8"}
    for k in bsmr.TUNING_ENV.values():
        monkeypatch.delenv(k, raising=False)
    assert bsmr.tuning_from_env() == {}
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    from_c = bsmr.tuning_from_env()
    from_py = bsmr.tuning_from_env(env)
    assert from_py == {"tile_min_f32": 0, "out_staged": 1, "orig_rows": -1,
                       "piece_weight": 2.5, "l2_range_kb": 64, "diag": 8}
    # orig_rows "auto" equals the default (-1), so the C parser reports no change for it
    assert from_c == {k: v for k, v in from_py.items() if k != "orig_rows"}
    with pytest.raises(bsmr.BsmrError):
        bsmr._tuning_struct({"no_such_knob": 1})


def test_tuning_defaults_and_struct_size():
    """bsmr_tuning_default fills exactly the ctypes mirror of the (ABI 13) tuning struct, every
    knob at its "keep the measured default" value; col_blocks (the column-block launch) is -1."""
    n = ctypes.sizeof(bsmr.Tuning)
    buf = (ctypes.c_uint8 * (n + 32))(*([0xAB] * (n + 32)))
    bsmr.lib().bsmr_tuning_default(ctypes.cast(buf, ctypes.POINTER(bsmr.Tuning)))
    assert bytes(buf[n:]) == b"\xab" * 32
    t = bsmr.Tuning.from_buffer(buf)
    assert t.diag == 0 and t.col_blocks == -1 and t.piece_balance == -1 and t.ptile == -1
    assert [f for f, _ in bsmr.Tuning._fields_][-1] == "col_blocks"
    assert [f for f, _ in bsmr.PlanStats._fields_][-1] == "rb_col_blocks"


def test_col_blocks_env_values(monkeypatch):
    """BSMR_COL_BLOCKS takes 0 / 1 / 2 (never, always, the wide-pattern piece rule) through both
    the library's parser and the Python mapping."""
    for k in bsmr.TUNING_ENV.values():
        monkeypatch.delenv(k, raising=False)
    for v in ("0", "1", "2"):
        monkeypatch.setenv("BSMR_COL_BLOCKS", v)
        assert bsmr.tuning_from_env() == {"col_blocks": int(v)}
        assert bsmr.tuning_from_env({"BSMR_COL_BLOCKS": v}) == {"col_blocks": int(v)}
