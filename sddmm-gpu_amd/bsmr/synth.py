"""Synthetic sparse patterns (host-side input generation, numpy).

Two families:

* Exact rebuilds of SuiteSparse matrices that appear in the reference's published logs and are
  defined by a formula (Trefethen_20000/20000b, mycielskian14/15/16). They reproduce what the
  reference loader (Matrix.cpp:398-480) builds from the SuiteSparse ``.mtx`` files: symmetric
  files store the lower triangle only and the loader does not mirror it, entries are listed
  column by column, so every CSR row holds its lower-triangle columns in ascending order.
* Seeded stand-ins for the BASELINE.json configs whose files are absent:
  nips_like, cop20k_A_like, reddit_like, dlmc_like.

All return (M, N, rowptr uint32[M+1], colidx uint32[nnz]).
"""
import numpy as np


def _csr_from_coo(M, N, rows, cols):
    rows = np.asarray(rows, dtype=np.int64)
    cols = np.asarray(cols, dtype=np.int64)
    order = np.lexsort((cols, rows))
    rows = rows[order]
    cols = cols[order]
    rowptr = np.zeros(M + 1, dtype=np.int64)
    np.add.at(rowptr, rows + 1, 1)
    rowptr = np.cumsum(rowptr)
    return M, N, rowptr.astype(np.uint32), cols.astype(np.uint32)


def trefethen(n):
    """Trefethen_<n>: primes on the diagonal, ones where |i-j| is a power of two (lower triangle)."""
    rows = [np.arange(n)]
    cols = [np.arange(n)]
    p = 1
    while p < n:
        r = np.arange(p, n)
        rows.append(r)
        cols.append(r - p)
        p <<= 1
    return _csr_from_coo(n, n, np.concatenate(rows), np.concatenate(cols))


def mycielskian(k):
    """mycielskian<k>: A_{j+1} = [A A 0; A 0 e; 0 e' 0] from A_2 = K_2; lower triangle stored."""
    n = 2
    ei = np.array([1], dtype=np.int64)  # edges as (i > j)
    ej = np.array([0], dtype=np.int64)
    for _ in range(k - 2):
        # v_i ~ u_j and v_j ~ u_i for each edge (i, j); u_i ~ w
        ni = np.concatenate([ei, n + ej, n + ei, np.full(n, 2 * n)])
        nj = np.concatenate([ej, ei, ej, n + np.arange(n)])
        ei = np.maximum(ni, nj)
        ej = np.minimum(ni, nj)
        n = 2 * n + 1
    return _csr_from_coo(n, n, ei, ej)


SUITESPARSE_REBUILDS = {
    "Trefethen_20000": lambda: trefethen(20000),
    "Trefethen_20000b": lambda: trefethen(19999),
    "mycielskian14": lambda: mycielskian(14),
    "mycielskian15": lambda: mycielskian(15),
    "mycielskian16": lambda: mycielskian(16),
}


def random_rows(M, N, nnz_per_row, seed, zipf=None, empty_frac=0.0):
    """Rows with nnz_per_row distinct columns (Poisson around a scalar, or an explicit
    per-row count array); Zipf-popular columns when zipf is set."""
    rng = np.random.default_rng(seed)
    if np.isscalar(nnz_per_row):
        counts = rng.poisson(nnz_per_row, size=M).clip(1, N)
    else:
        counts = np.asarray(nnz_per_row).clip(0, N)
    if empty_frac > 0:
        counts[rng.random(M) < empty_frac] = 0
    if zipf is not None:
        w = 1.0 / np.arange(1, N + 1) ** zipf
        w /= w.sum()
        perm = rng.permutation(N)
    rows, cols = [], []
    for r in range(M):
        c = int(counts[r])
        if c == 0:
            continue
        if zipf is not None:
            pick = perm[rng.choice(N, size=c, replace=False, p=w)]
        else:
            pick = rng.choice(N, size=c, replace=False)
        rows.append(np.full(len(pick), r))
        cols.append(pick)
    return _csr_from_coo(M, N, np.concatenate(rows), np.concatenate(cols))


def nips_like(seed=20250801):
    """C1/C2 stand-in: 1,500 x 12,419 with exactly 746,316 nnz (the UCI NIPS docword shape),
    log-normal document lengths, Zipf(1.1) word popularity."""
    M, N, target = 1500, 12419, 746316
    rng = np.random.default_rng(seed)
    lens = rng.lognormal(mean=np.log(440), sigma=0.5, size=M)
    lens = np.clip(np.round(lens * (target / lens.sum())), 8, N // 2).astype(np.int64)
    diff = target - int(lens.sum())
    step = 1 if diff > 0 else -1
    i = 0
    while diff != 0:
        j = i % M
        if 8 <= lens[j] + step <= N // 2:
            lens[j] += step
            diff -= step
        i += 1
    return random_rows(M, N, lens, seed + 1, zipf=1.1)


def banded_fem_like(n, nnz_per_row, seed, band=64, target=None):
    """cop20k_A-like: banded FEM block structure plus a few random long-range couplings.
    nnz_per_row draws per row (80 % inside the band, 20 % anywhere); duplicates merge, so the
    pattern holds fewer entries than n * nnz_per_row. target: top the pattern up with further
    draws of the same mix, then keep a seeded sample of exactly `target` distinct entries."""
    rng = np.random.default_rng(seed)
    k_band = int(nnz_per_row * 0.8)
    k_rand = nnz_per_row - k_band

    def draw(r, kb, kr):
        off = rng.integers(-band, band + 1, size=(len(r), kb))
        c = np.clip(r[:, None] + off, 0, n - 1)
        c2 = rng.integers(0, n, size=(len(r), kr))
        cc = np.concatenate([c, c2], axis=1)
        return np.repeat(r, cc.shape[1]).astype(np.int64) * n + cc.reshape(-1)

    keys = [draw(np.arange(r0, min(n, r0 + 4096)), k_band, k_rand) for r0 in range(0, n, 4096)]
    key = np.unique(np.concatenate(keys))
    while target is not None and len(key) < target:
        # one more draw per row of the same 4:1 band / random mix until enough distinct entries
        r = rng.integers(0, n, size=max(1024, 2 * (target - len(key))))
        extra = draw(r, 1, 0)
        rnd = rng.random(len(r)) < k_rand / nnz_per_row
        extra[rnd] = r[rnd].astype(np.int64) * n + rng.integers(0, n, size=int(rnd.sum()))
        key = np.unique(np.concatenate([key, extra]))
    if target is not None and len(key) > target:
        key = np.sort(rng.choice(key, size=target, replace=False))
    return _csr_from_coo(n, n, key // n, key % n)


def cop20k_like(seed=20250802):
    """C3 stand-in: 121,192 x 121,192 FEM-like pattern with exactly 2,624,331 stored entries
    (cop20k_A's full pattern, 21.65 per row)."""
    return banded_fem_like(121192, 22, seed, band=48, target=2_624_331)


_synth_lib = None


def _synth():
    """lib/libbsmr_synth.so (synth/chung_lu.cpp): the multi-threaded graph generator."""
    global _synth_lib
    if _synth_lib is None:
        import ctypes as C
        import os

        path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib",
                            "libbsmr_synth.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} is missing (run `make -C sddmm-gpu_amd`)")
        L = C.CDLL(path)
        u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
        L.bsmr_synth_chung_lu.argtypes = [C.c_uint32, C.c_uint64, C.c_uint64, C.c_double, u32p,
                                          u32p]
        _synth_lib = L
    return _synth_lib


def chung_lu(n, nnz_target, seed, exponent=2.2):
    """Symmetric power-law graph (Chung-Lu): endpoints drawn with probability proportional to
    w_i = (i+1)^(-1/(exponent-1)) over a seeded relabelling of the nodes; self loops dropped,
    each undirected edge kept once, then both directions stored with ascending columns per row.
    Draws continue until nnz_target / 2 distinct edges exist (the heavy rows repeat pairs, so a
    fixed number of draws falls short), and exactly that many are kept (the smallest seeded
    hashes): the result holds nnz_target stored entries (rounded down to even). Generated in C++
    over fixed (seed, round, chunk) random streams (synth/chung_lu.cpp: the same pattern for any
    thread count; reddit_like x1 in ~10 s instead of ~150 s for the numpy form of round 2)."""
    nnz = int(nnz_target) // 2 * 2
    rowptr = np.empty(n + 1, np.uint32)
    colidx = np.empty(nnz, np.uint32)
    st = _synth().bsmr_synth_chung_lu(int(n), nnz, int(seed), float(exponent), rowptr, colidx)
    if st != 0:
        raise ValueError(f"chung_lu: {n} nodes cannot hold {nnz} stored entries")
    return n, n, rowptr, colidx


def reddit_like(scale=1.0, seed=20250803):
    """C4 stand-in: 232,965-node power-law graph with 232,000,000 stored entries at scale 1
    (BASELINE.json quotes ~232M nnz: the public Reddit graph's 114,615,892 undirected edges stored
    in both directions, ~229M). scale < 1 shrinks the nodes by scale and the entries by scale^2."""
    n = max(1024, int(232965 * scale))
    return chung_lu(n, int(232_000_000 * scale * scale), seed)


def stack_copies(M, N, rowptr, colidx, copies, seed=20251016):
    """Weak-scaling workload: `copies` row blocks, block b = the pattern with its columns relabelled
    by a random permutation of [0, N) (block 0 unchanged), so the blocks' rows are as unlike each
    other as the pattern's own rows and each block carries the pattern's work. Every row's columns
    are re-sorted after the relabelling, as in a .mtx file loaded by the reference (ascending within
    a row): unsorted rows interleave the XCD column ranges inside each row's CSR segment, so every
    128-byte line of P would be written by several L2s (one copy: 14.9 vs 11.2 us,
    tools/copy_order_check.py). copies = 1 returns the pattern itself."""
    rowptr = np.asarray(rowptr, dtype=np.uint32)
    colidx = np.asarray(colidx, dtype=np.uint32)
    if copies == 1:
        return M, N, rowptr, colidx
    rng = np.random.default_rng(seed)
    nnz = int(rowptr[-1])
    rp = np.empty(copies * M + 1, dtype=np.uint64)
    ci = np.empty(copies * nnz, dtype=np.uint32)
    rp[0] = 0
    for b in range(copies):
        perm = np.arange(N, dtype=np.uint32) if b == 0 else rng.permutation(N).astype(np.uint32)
        rp[1 + b * M: 1 + (b + 1) * M] = rowptr[1:].astype(np.uint64) + b * nnz
        cb = perm[colidx]
        for r in range(M):  # ascending columns within each row
            cb[rowptr[r]:rowptr[r + 1]].sort()
        ci[b * nnz:(b + 1) * nnz] = cb
    if rp[-1] >= 2 ** 32:
        raise ValueError("stack_copies: more than 2^32 stored entries")
    return copies * M, N, rp.astype(np.uint32), ci


def dlmc_like(kind="uniform", seed=7):
    """C5 stand-in: 2,048 x 2,048 transformer mask at 90 % sparsity, uniform or 16x16 blocks."""
    if kind == "uniform":
        return uniform_mask(2048, 0.1, seed)
    return block_mask(2048, 16, 0.1, seed)


def block_mask(n, block, density, seed):
    """DLMC-like 2-D mask: 16x16 (block) structured at the given block density."""
    rng = np.random.default_rng(seed)
    nb = n // block
    mask = rng.random((nb, nb)) < density
    br, bc = np.nonzero(mask)
    rr = (br[:, None] * block + np.arange(block)[None, :])
    cc = (bc[:, None] * block + np.arange(block)[None, :])
    rows = np.repeat(rr, block, axis=1).reshape(-1)
    cols = np.tile(cc, (1, block)).reshape(-1)
    return _csr_from_coo(n, n, rows, cols)


def uniform_mask(n, density, seed):
    rng = np.random.default_rng(seed)
    total = int(n * n * density)
    key = np.unique(rng.integers(0, n * n, size=int(total * 1.05)))[:total]
    return _csr_from_coo(n, n, key // n, key % n)


def write_mtx(path, M, N, rowptr, colidx, symmetric_header=False):
    """Write a Matrix Market coordinate pattern file (1-based) in CSR order."""
    nnz = int(rowptr[-1])
    rows = np.repeat(np.arange(M, dtype=np.int64), np.diff(rowptr.astype(np.int64)))
    with open(path, "w") as f:
        kind = "symmetric" if symmetric_header else "general"
        f.write(f"%%MatrixMarket matrix coordinate pattern {kind}\n")
        f.write(f"{M} {N} {nnz}\n")
        data = np.stack([rows + 1, colidx.astype(np.int64) + 1], axis=1)
        np.savetxt(f, data, fmt="%d")


def write_smtx(path, M, N, rowptr, colidx):
    """Write a DLMC .smtx file: header "M, N, nnz" words, one line of row offsets, one of column
    indices (the format CSR::initializeFromSmtxFile reads, src/Matrix.cpp:296-371)."""
    with open(path, "w") as f:
        f.write(f"{M} {N} {int(rowptr[-1])}\n")
        f.write(" ".join(str(int(x)) for x in rowptr) + "\n")
        f.write(" ".join(str(int(x)) for x in colidx) + "\n")


def write_snap(path, M, rowptr, colidx, id_base=1):
    """Write a square pattern as a SNAP edge list ("# Nodes:"/"# Edges:" header, "from\\tto" per
    line). Node ids are id_base + index; the loader renumbers them by first appearance, so the
    loaded matrix is a symmetric permutation of this one (CSR::initializeFromGraphDataset)."""
    nnz = int(rowptr[-1])
    rows = np.repeat(np.arange(M, dtype=np.int64), np.diff(rowptr.astype(np.int64)))
    with open(path, "w") as f:
        f.write(f"# Directed graph: {path}\n# Nodes: {M} Edges: {nnz}\n# FromNodeId\tToNodeId\n")
        data = np.stack([rows + id_base, colidx.astype(np.int64) + id_base], axis=1)
        np.savetxt(f, data, fmt="%d", delimiter="\t")
