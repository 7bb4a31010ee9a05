"""CPU check of the clustering candidate filter's bound (sddmm-gpu_amd/csrc/cluster_filter.hip).

The chain accepts a row into a cluster iff mn (1 + alpha) > alpha S with
mn = sum_i min(a_i / nr, b_i / nc), S = S1R / nr + S1C / nc (rowReordering.cu:235-293, restated
in oracle.cpp similarity_exact). The filter clears the bit of a pair only when
G (1 + alpha) 1.01 <= alpha (u_q + u_p) sqrt(n_q) sqrt(n_p), G = <sqrt a, sqrt b> from fp16 values
rounded up and accumulated in fp32. These tests restate that arithmetic in numpy and check that a
cleared bit is always a true reject (no accept is ever skipped), on random count vectors shaped
like the reference's block encodings, including the pairs closest to alpha.
"""
import zlib

import numpy as np
import pytest


def sqrt_up_f16(c):
    """sqrt of the counts as fp16 rounded up (k_filter_x)."""
    f = np.sqrt(c.astype(np.float32)) * np.float32(1.000001)
    h = f.astype(np.float16)
    low = h.astype(np.float32) < f
    h[low] = np.nextafter(h[low], np.float16(np.inf))
    return h


def filter_bit(a, b, alpha):
    """The filter's verdict for one pair (True: the chain must evaluate it)."""
    SR, SC = np.uint32((a.astype(np.uint64) ** 2).sum()), np.uint32((b.astype(np.uint64) ** 2).sum())
    if SR == 0 or SC == 0:
        return True
    nr, nc = np.sqrt(np.float32(SR)), np.sqrt(np.float32(SC))
    uq, up = np.float32(a.sum()) / nr, np.float32(b.sum()) / nc
    # fp32 accumulation of fp16 products, in the worst order for a lower result (ascending)
    prod = np.sort(sqrt_up_f16(a).astype(np.float32) * sqrt_up_f16(b).astype(np.float32))
    G = np.float32(0)
    for v in prod:
        G = np.float32(G + v)
    c1 = np.float32((1 + alpha) * 1.01)
    rhs = np.float32(alpha) * (uq + up) * np.sqrt(nr) * np.sqrt(nc)
    return bool(G * c1 > rhs)


def accepts(a, b, alpha):
    """The chain's decision, in double from the same fp32 norms (the estimate of plan.hip
    cl_verdict; the exact fp32 tree differs by < 3e-6, inside the filter's 1 % margin)."""
    SR, SC = int((a.astype(np.int64) ** 2).sum()), int((b.astype(np.int64) ** 2).sum())
    if SR == 0 and SC == 0:
        return 1.0 > alpha
    if SR == 0 or SC == 0:
        return 0.0 > alpha
    nr, nc = float(np.sqrt(np.float32(SR))), float(np.sqrt(np.float32(SC)))
    mn = np.minimum(a / nr, b / nc).sum()
    mx = a.sum() / nr + b.sum() / nc - mn
    return mn / mx > alpha


def random_pair(rng, nb, kind):
    if kind == "binary":  # graph rows: most blocks hold one entry
        a = (rng.random(nb) < 0.1).astype(np.int64)
        b = (rng.random(nb) < 0.1).astype(np.int64)
    elif kind == "counts":
        a = rng.poisson(0.4, nb) * (rng.random(nb) < 0.3)
        b = rng.poisson(0.4, nb) * (rng.random(nb) < 0.3)
    elif kind == "similar":  # b a perturbed copy of a: sims spread around alpha
        a = rng.poisson(1.5, nb) * (rng.random(nb) < 0.2)
        b = np.maximum(a + rng.integers(-1, 2, nb) * (rng.random(nb) < 0.5), 0)
    else:  # hub: wide range of counts (up to the block width)
        a = rng.integers(0, 38, nb) * (rng.random(nb) < 0.05)
        b = rng.integers(0, 38, nb) * (rng.random(nb) < 0.05)
    return a, b


@pytest.mark.parametrize("kind", ["binary", "counts", "similar", "hub"])
@pytest.mark.parametrize("alpha", [0.01, 0.1, 0.3, 0.7, 0.9])
def test_cleared_bit_is_a_true_reject(kind, alpha):
    rng = np.random.default_rng(zlib.crc32(f"{kind}:{alpha}".encode()))
    skipped = 0
    for _ in range(300):
        a, b = random_pair(rng, int(rng.integers(8, 400)), kind)
        if not filter_bit(a, b, alpha):
            skipped += 1
            assert not accepts(a, b, alpha), (a.tolist(), b.tolist())
    # the filter does reject (it is not vacuous) where the pairs are far from alpha
    if kind == "binary" and alpha >= 0.3:
        assert skipped > 0


def test_bound_is_exact_for_binary_counts():
    """0/1 counts: min(1/nr, 1/nc) <= 1/sqrt(nr nc) per common block, so U >= mn, with equality
    when the two norms are equal (rows of equal block count, the common case next to each other
    in the dispersion order)."""
    rng = np.random.default_rng(5)
    for _ in range(100):
        a = (rng.random(200) < 0.2).astype(np.int64)
        b = (rng.random(200) < 0.2).astype(np.int64)
        if a.sum() == 0 or b.sum() == 0:
            continue
        nr, nc = np.sqrt(float((a ** 2).sum())), np.sqrt(float((b ** 2).sum()))
        mn = np.minimum(a / nr, b / nc).sum()
        U = np.sqrt(a * b).sum() / np.sqrt(nr * nc)
        # min(1/nr, 1/nc) vs 1/sqrt(nr nc): equal only for nr == nc; U >= mn always
        assert U >= mn - 1e-12


def test_triangle_row_offsets():
    """fbits_row_offset (plan_kernels.hpp): row q starts after rows 0..q-1 of W - r/32 words."""
    for M in (1, 31, 32, 33, 100, 1000):
        W = (M + 31) // 32

        def off(q):
            a, b = q >> 5, q & 31
            return q * W - (16 * a * (a - 1) + a * b)
        acc = 0
        for q in range(M + 1):
            assert off(q) == acc
            acc += W - q // 32
