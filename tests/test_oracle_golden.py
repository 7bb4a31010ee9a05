"""Pin the CPU oracle against the reference's own published logs (golden vectors).

For every matrix of the reference logs that can be rebuilt exactly (tests/golden/, made by
tools/extract_reference_log_stats.py), the oracle's row reordering, column split and tile layout
must reproduce every statistic the reference printed, for all alpha x delta settings and all
four K values of the sweep (K only changes the sparse launch shape).
"""
import functools

import numpy as np
import pytest

import oracle_lib as O
from golden_common import (ALPHAS, DELTAS, REF_FREE_MEM, compare, expected_from_stats, matrix,
                           record)


@functools.lru_cache(maxsize=None)
def oracle_csr(name):
    M, N, rp, ci = matrix(name)
    return O.CSR.from_arrays(M, N, rp, ci)


@functools.lru_cache(maxsize=None)
def oracle_rows(name, alpha):
    c = oracle_csr(name)
    bs = O.block_size(c.M, c.N, REF_FREE_MEM)
    return O.row_reorder(c, np.float32(alpha), bs)


def oracle_stats(name, alpha, delta):
    rows, ncl, _ = oracle_rows(name, alpha)
    p = O.Plan(oracle_csr(name), rows, ncl, np.float32(delta))
    s = p.stats()
    return {
        "numRowPanels": s["numRowPanels"], "numClusters": s["numClusters"],
        "numDenseBlock": s["numDenseBlock"], "averageDensity": s["averageDensity"],
        "originalNumDenseBlock": s["originalNumDenseBlock"],
        "originalAverageDensity": s["originalAverageDensity"],
        "numDenseThreadBlocks": s["numDenseThreadBlocks"],
        "numSparseThreadBlocks": s["numSparseThreadBlocks"],
        "numDenseData": s["numDenseData"], "numSparseData": s["numSparseData"],
        "maxDense": s["maxNumDenseColBlocksInRowPanel"],
        "rphmSparseTB": s["rphmNumSparseThreadBlocks"],
    }


def _check(name, alpha):
    bad = {}
    for delta in DELTAS:
        s = oracle_stats(name, alpha, delta)
        for K in (32, 64, 128, 256):
            diff = compare(expected_from_stats(s, K), record(name, alpha, delta, K))
            if diff:
                bad[(delta, K)] = diff
    assert not bad, bad


def test_matrix_rebuilds_match_logged_shapes():
    for name in ("Trefethen_20000", "Trefethen_20000b", "mycielskian14", "mycielskian15",
                 "mycielskian16"):
        M, N, rp, ci = matrix(name)
        r = record(name, 0.3, 0.3)
        assert (M, N, len(ci)) == (r["M"], r["N"], r["NNZ"])
        total = M * N
        sp = np.float32(1.0) - np.float32(len(ci)) / np.float32(total)
        assert f"{np.floor(sp * np.float32(10000)) / 100.0:.2f}%" == r["sparsity"]


@pytest.mark.parametrize("alpha", ALPHAS)
@pytest.mark.parametrize("name", ["Trefethen_20000", "Trefethen_20000b", "mycielskian14"])
def test_oracle_matches_reference_logs(name, alpha):
    _check(name, alpha)


@pytest.mark.parametrize("alpha", [0.1, 0.3, 0.5, 0.7])
def test_oracle_matches_reference_logs_mycielskian15(alpha):
    _check("mycielskian15", alpha)


@pytest.mark.parametrize("alpha", [0.1, 0.3])
def test_oracle_matches_reference_logs_mycielskian16(alpha):
    _check("mycielskian16", alpha)


@pytest.mark.slow
@pytest.mark.parametrize("name,alpha", [("mycielskian15", 0.9), ("mycielskian16", 0.5),
                                        ("mycielskian16", 0.7), ("mycielskian16", 0.9)])
def test_oracle_matches_reference_logs_long(name, alpha):
    _check(name, alpha)
