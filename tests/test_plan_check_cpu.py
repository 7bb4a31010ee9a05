"""CPU tests of the product's structural plan check (bsmr_check_rphm_arrays, the host half of
bsmr_plan_check): the reference's check_rphm (src/BSMR.cpp:932-953 -> 444-824), run under VALIDATE
before checkSddmm (src/sddmm.cu:34-38).

The oracle's plans (tests/oracle_lib: the CPU restatement pinned against the reference logs) must
pass at every delta, including delta = 0 (every 16-column group dense, padded groups too) and 1.1
(no dense group); each corruption of one array must fail with the reference's message for that
stage ("Error! The row reordering is incorrect!", "... col reordering ...", "... rphm ...").
"""
import numpy as np
import pytest

import oracle_lib as O
import bsmr
from bsmr import synth
from gpu_util import PLAN_ARRAYS

FREE = 288 * 1024 ** 3


def _oracle_arrays(M, N, rp, ci, alpha, delta):
    c = O.CSR.from_arrays(M, N, rp, ci)
    rows, ncl, _ = O.row_reorder(c, np.float32(alpha), O.block_size(M, N, FREE))
    op = O.Plan(c, rows, ncl, np.float32(delta))
    return {k: op.array(k).copy() for k in PLAN_ARRAYS}


CASES = {
    "ragged_empty_rows": lambda: synth.random_rows(300, 1000, 25, seed=1, empty_frac=0.1),
    "zipf": lambda: synth.random_rows(517, 4000, 60, seed=2, zipf=1.1),
    "blocky": lambda: synth.block_mask(256, 16, 0.2, seed=4),
    "trefethen": lambda: synth.trefethen(700),
    "mycielskian8": lambda: synth.mycielskian(8),
}


@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("delta", [0.0, 0.3, 1.1])
def test_oracle_plans_pass(name, delta, capfd):
    M, N, rp, ci = CASES[name]()
    arr = _oracle_arrays(M, N, rp, ci, 0.3, delta)
    ok, msg = bsmr.check_rphm_arrays(M, N, rp, ci, arr, delta)
    err = capfd.readouterr().err
    assert ok and msg == "" and err == "", (msg, err)


def _first_dense_panel(arr):
    dco = arr["denseColOffsets"]
    for q in range(len(dco) - 1):
        if dco[q + 1] - dco[q] >= 32:
            return q
    raise AssertionError("no panel with two dense tiles")


def _corrupt(kind, arr, M, N, rp, ci):
    a = {k: v.copy() for k, v in arr.items()}
    if kind == "row_duplicated":
        a["reorderedRows"][1] = a["reorderedRows"][0]
        return a, "Error! Row is duplicated!", "Error! The row reordering is incorrect!"
    if kind == "row_missing_empty_stored":
        empty = np.nonzero(np.diff(rp) == 0)[0]
        a["reorderedRows"][3] = empty[0]
        return a, "Error! Empty row is stored!", "Error! The row reordering is incorrect!"
    if kind == "dense_col_order":
        q = _first_dense_panel(a)
        d0 = a["denseColOffsets"][q]
        dc = a["denseCols"]
        # the first and the last real dense column of the panel swap places (counts differ)
        j = d0 + 15
        dc[d0], dc[j] = dc[j], dc[d0]
        return a, "Error! The order of column indexes in the row panel is incorrect!", \
            "Error! The col reordering is incorrect!"
    if kind == "sparse_col_not_in_panel":
        s = a["sparseCols"]
        sco = a["sparseColOffsets"]
        q = next(q for q in range(len(sco) - 1) if sco[q + 1] > sco[q] and s[sco[q]] != N)
        rows = a["reorderedRows"][16 * q:16 * q + 16]
        used = set(np.concatenate([ci[rp[r]:rp[r + 1]] for r in rows]).tolist())
        s[sco[q]] = next(c for c in range(N) if c not in used)
        return a, "Error! Column index not in current row panel!", \
            "Error! The col reordering is incorrect!"
    if kind == "block_value_wrong":
        bv = a["blockValues"]
        i = int(np.nonzero(bv != 0xFFFFFFFF)[0][5])
        bv[i] = bv[i] + 1 if bv[i] + 1 < len(ci) else bv[i] - 1
        return a, "Error! The block value is incorrect!", "Error! The rphm is incorrect!"
    if kind == "block_value_missing":
        bv = a["blockValues"]
        i = int(np.nonzero(bv != 0xFFFFFFFF)[0][7])
        bv[i] = 0xFFFFFFFF
        return a, "Error! Missing value!", "Error! The rphm is incorrect!"
    if kind == "sparse_value_wrong":
        sv = a["sparseValues"]
        sv[2], sv[3] = sv[3], sv[2]
        return a, "Error! The sparse value is incorrect!", "Error! The rphm is incorrect!"
    raise KeyError(kind)


@pytest.mark.parametrize("kind", ["row_duplicated", "row_missing_empty_stored", "dense_col_order",
                                  "sparse_col_not_in_panel", "block_value_wrong",
                                  "block_value_missing", "sparse_value_wrong"])
def test_corrupted_plan_fails_with_reference_text(kind, capfd):
    M, N, rp, ci = synth.random_rows(400, 300, 40, seed=5, zipf=1.3, empty_frac=0.05)
    arr = _oracle_arrays(M, N, rp, ci, 0.3, 0.3)
    assert bsmr.check_rphm_arrays(M, N, rp, ci, arr, 0.3, verbose=False)[0]
    bad, line, summary = _corrupt(kind, arr, M, N, rp, ci)
    ok, msg = bsmr.check_rphm_arrays(M, N, rp, ci, bad, 0.3)
    err = capfd.readouterr().err
    assert not ok
    assert line in msg and line in err, (msg, err)
    assert summary in err, err


def test_delta_mismatch_is_caught(capfd):
    """A plan built for delta = 0.3 checked against delta = 0.5: the dense prefix no longer matches
    ceil(delta * 256) (colReordering.cu:244-271)."""
    M, N, rp, ci = synth.random_rows(400, 300, 40, seed=5, zipf=1.3)
    arr = _oracle_arrays(M, N, rp, ci, 0.3, 0.3)
    ok, msg = bsmr.check_rphm_arrays(M, N, rp, ci, arr, 0.5)
    err = capfd.readouterr().err
    assert not ok and "does not match delta" in msg
    assert "Error! The col reordering is incorrect!" in err


@pytest.mark.parametrize("kind", ["colidx_past_N", "rowptr_decreasing", "rowptr_past_nnz"])
def test_malformed_csr_is_rejected_before_checking(kind):
    """bsmr_check_rphm_arrays takes untrusted host arrays: a column index >= N or a rowptr that is
    not non-decreasing within [0, nnz] is refused with BSMR_ERR_INVALID before any check indexes
    per-column or per-entry vectors with it (colidx == N + 5 used to write past them)."""
    M, N, rp, ci = synth.random_rows(200, 300, 20, seed=6)
    arr = _oracle_arrays(M, N, rp, ci, 0.3, 0.3)
    rp, ci = rp.astype(np.uint32).copy(), ci.astype(np.uint32).copy()
    if kind == "colidx_past_N":
        ci[len(ci) // 2] = N + 5
        want = "is not below N"
    elif kind == "rowptr_decreasing":
        rp[50] = rp[52] + 1
        want = "rowptr is not non-decreasing"
    else:
        rp[10] = len(ci) + 7
        want = "rowptr is not non-decreasing"
    with pytest.raises(bsmr.BsmrError) as ei:
        bsmr.check_rphm_arrays(M, N, rp, ci, arr, 0.3, verbose=False)
    assert "status 1" in str(ei.value) and want in str(ei.value), str(ei.value)
