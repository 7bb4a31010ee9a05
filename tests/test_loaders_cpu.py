"""The .smtx (DLMC) and SNAP .txt loaders and the suffix dispatch (SURVEY.md §8(f) row 2,
src/Matrix.cpp:279-371, 482-575): the product loaders (C ABI) against the oracle restatement on
generated files, including the rejection cases. CPU only."""
import numpy as np
import pytest

import bsmr
import oracle_lib as O


def write(path, text):
    path.write_bytes(text.encode())
    return str(path)


def both(path):
    g = bsmr.load(path)
    o = O.CSR.load(path)
    return g, o


def assert_same(g, o):
    assert g is not None and o is not None
    assert (g.M, g.N, g.nnz) == (o.M, o.N, o.nnz)
    grp, gci = g.rowptr, g.colidx
    orp, oci, ov = o.arrays()
    np.testing.assert_array_equal(grp, orp)
    np.testing.assert_array_equal(gci, oci)
    np.testing.assert_array_equal(g.values, ov)


def smtx_text(M, N, rowptr, colidx, comments=("% dlmc",), sep=" ", eol="\n"):
    lines = list(comments) + [f"{M}, {N}, {len(colidx)}".replace(", ", sep),
                              sep.join(str(x) for x in rowptr), sep.join(str(x) for x in colidx)]
    return eol.join(lines) + eol


def random_pattern(M, N, density, seed):
    rng = np.random.default_rng(seed)
    rows = []
    for _ in range(M):
        k = rng.binomial(N, density)
        rows.append(rng.choice(N, size=k, replace=False))  # unsorted: file order must be kept
    rowptr = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.uint32)
    colidx = np.concatenate(rows).astype(np.uint32) if rowptr[-1] else np.zeros(0, np.uint32)
    return rowptr, colidx


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_smtx_random_matches_oracle(tmp_path, seed):
    rp, ci = random_pattern(37 + seed, 50 + 3 * seed, 0.2, seed)
    p = write(tmp_path / "m.smtx", smtx_text(len(rp) - 1, 50 + 3 * seed, rp, ci))
    g, o = both(p)
    assert_same(g, o)
    np.testing.assert_array_equal(g.colidx, ci)  # file order inside rows
    assert (g.values == 1).all()


@pytest.mark.parametrize("sep,eol", [("\t", "\n"), (" ", "\r\n")])
def test_smtx_separators(tmp_path, sep, eol):
    rp, ci = random_pattern(20, 30, 0.3, 9)
    p = write(tmp_path / "m.smtx", smtx_text(20, 30, rp, ci, ("% a", "% b"), sep, eol))
    assert_same(*both(p))


@pytest.mark.parametrize("case", ["nnz0", "short_rowptr", "short_cols", "dup_in_row", "col_oob",
                                  "bad_offsets", "garbage_header"])
def test_smtx_rejections(tmp_path, case):
    texts = {
        "nnz0": "3 3 0\n0 0 0 0\n\n",
        "short_rowptr": "3 3 2\n0 1 2\n0 1\n",
        "short_cols": "3 3 3\n0 1 2 3\n0 1\n",
        "dup_in_row": "2 3 3\n0 2 3\n1 1 0\n",
        "col_oob": "2 3 2\n0 1 2\n0 3\n",
        "bad_offsets": "2 3 2\n0 2 1\n0 1\n",
        "garbage_header": "x 3 2\n0 1 2\n0 1\n",
    }
    p = write(tmp_path / "m.smtx", texts[case])
    g, o = both(p)
    assert g is None and o is None
    assert bsmr.lib().bsmr_last_error()


def snap_text(edges, nodes=None, nedges=None, same_line=False, values=False):
    n = nodes if nodes is not None else len({x for e in edges for x in e})
    m = nedges if nedges is not None else len(edges)
    head = ["# Directed graph (each unordered pair of nodes is saved once): test.txt"]
    head += [f"# Nodes: {n} Edges: {m}"] if same_line else [f"# Nodes: {n}", f"# Edges: {m}"]
    head.append("# FromNodeId\tToNodeId")
    body = [f"{a}\t{b}" + (f"\t{0.5 * i}" if values else "") for i, (a, b) in enumerate(edges)]
    return "\n".join(head + body) + "\n"


@pytest.mark.parametrize("same_line,values", [(False, False), (True, True)])
def test_snap_renumbers_by_first_appearance(tmp_path, same_line, values):
    edges = [(100, 7), (7, 42), (42, 100), (5, 7), (100, 5), (7, 100)]
    p = write(tmp_path / "g.txt", snap_text(edges, same_line=same_line, values=values))
    g, o = both(p)
    assert_same(g, o)
    # ids: 100->0, 7->1, 42->2, 5->3; rows stably sorted
    assert (g.M, g.N, g.nnz) == (4, 4, 6)
    np.testing.assert_array_equal(g.rowptr, [0, 2, 4, 5, 6])
    np.testing.assert_array_equal(g.colidx, [1, 3, 2, 0, 0, 1])


def test_snap_random_matches_oracle(tmp_path):
    rng = np.random.default_rng(5)
    pairs = set()
    while len(pairs) < 400:
        a, b = (int(x) for x in rng.integers(0, 10 ** 6, 2)) if len(pairs) % 7 else (1, len(pairs))
        pairs.add((a, b))
    edges = list(pairs)
    text = snap_text(edges)
    text = text.replace(f"\n{edges[3][0]}\t", f"\n\n{edges[3][0]}\t", 1)  # a blank data line
    p = write(tmp_path / "g.txt", text)
    assert_same(*both(p))


@pytest.mark.parametrize("case", ["no_header", "too_many", "too_few", "too_big", "dup"])
def test_snap_rejections(tmp_path, case):
    e = [(1, 2), (2, 3), (3, 1)]
    texts = {
        "no_header": "1\t2\n2\t3\n",
        "too_many": snap_text(e, nedges=2),
        "too_few": snap_text(e, nedges=4),
        "too_big": snap_text(e, nodes=2),
        "dup": snap_text(e + [(2, 3)]),
    }
    p = write(tmp_path / "g.txt", texts[case])
    g, o = both(p)
    assert g is None and o is None


def test_dispatch(tmp_path):
    rp, ci = random_pattern(10, 10, 0.4, 3)
    lines = ["%%MatrixMarket matrix coordinate pattern general", f"10 10 {len(ci)}"]
    for r in range(10):
        for k in range(rp[r], rp[r + 1]):
            lines.append(f"{r + 1} {ci[k] + 1}")
    mtx = write(tmp_path / "m.mtx", "\n".join(lines) + "\n")
    smtx = write(tmp_path / "m.smtx", smtx_text(10, 10, rp, ci))
    a, b = bsmr.load(mtx), bsmr.load(smtx)
    np.testing.assert_array_equal(a.rowptr, b.rowptr)
    np.testing.assert_array_equal(a.colidx, b.colidx)
    assert bsmr.load(str(tmp_path / "m.csv")) is None
    assert O.CSR.load(str(tmp_path / "m.csv")) is None


@pytest.mark.parametrize("edges,nodes,msg", [
    ([(1, 2), (1, 2), (3, 4)], 2, "duplicate"),  # repeat (edge 1) before the first big id (edge 2)
    ([(1, 2), (3, 4), (1, 2)], 2, "too big"),    # big id (edge 1) before the repeat (edge 2)
])
def test_snap_first_offending_edge_decides(tmp_path, edges, nodes, msg):
    p = write(tmp_path / "g.txt", snap_text(edges, nodes=nodes))
    assert bsmr.load(p) is None
    assert msg in bsmr.lib().bsmr_last_error().decode()
    assert O.CSR.load(p) is None
