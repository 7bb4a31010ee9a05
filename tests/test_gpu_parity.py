"""GPU parity: the HIP plan builder and SDDMM kernels against the CPU oracle (through the C ABI).

* plan arrays (reorderedRows, dense/sparse columns, tile indices, residual lists): bit-exact;
* reorder statistics: equal to the reference's published logs (golden vectors);
* SDDMM values: checkData rule of the reference (|a-b| < 1e-5 or rel < 1e-3) against the
  oracle's host SDDMM (host.cpp:45-76 loop order), zero mismatches allowed.
"""
import functools

import numpy as np
import pytest

import oracle_lib as O
from bsmr import Plan, make_data, synth, tuning_from_env
from golden_common import (ALPHAS, DELTAS, REF_FREE_MEM, compare, expected_from_stats, matrix,
                           record)
from gpu_util import assert_plans_equal, half_values, oracle_plan, run_sddmm, torch_cuda

pytestmark = pytest.mark.gpu

FREE = 288 * 1024 ** 3


@functools.lru_cache(maxsize=None)
def small_cases():
    cases = {
        "ragged_empty_rows": synth.random_rows(300, 1000, 25, seed=1, empty_frac=0.1),
        "zipf": synth.random_rows(517, 4000, 60, seed=2, zipf=1.1),
        "wide_bs20": synth.random_rows(200, 120000, 300, seed=3),
        "blocky": synth.block_mask(512, 16, 0.15, seed=4),
        "trefethen_small": synth.trefethen(2000),
        "mycielskian10": synth.mycielskian(10),
    }
    return cases


@pytest.mark.parametrize("name", ["ragged_empty_rows", "zipf", "wide_bs20", "blocky",
                                  "trefethen_small", "mycielskian10"])
@pytest.mark.parametrize("alpha", [0.1, 0.3, 0.9])
def test_plan_bit_exact_small(name, alpha):
    M, N, rp, ci = small_cases()[name]
    gp = Plan(M, N, rp, ci, alpha=alpha, delta=0.3, free_mem_bytes=FREE)
    c, op, ncl = oracle_plan(M, N, rp, ci, alpha, 0.3, FREE)
    assert gp.stats()["num_clusters"] == ncl
    assert_plans_equal(gp, op)
    for delta in (0.0, 1.1, 0.5):
        gp.recolumn(delta)
        op2 = O.Plan(c, op.array("reorderedRows"), ncl, np.float32(delta))
        assert_plans_equal(gp, op2)


@pytest.mark.parametrize("name", ["zipf", "wide_bs20", "mycielskian10"])
def test_exact_similarity_mode_same_permutation(name):
    M, N, rp, ci = small_cases()[name]
    a = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE)
    b = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE, exact_similarity=True)
    assert b.stats()["exact_similarity_evals"] == b.stats()["total_similarity_evals"]
    assert np.array_equal(a.array("reorderedRows"), b.array("reorderedRows"))
    c = O.CSR.from_arrays(M, N, rp, ci)
    rows, ncl, _ = O.row_reorder(c, np.float32(0.3), O.block_size(M, N, FREE), exact_all=True)
    assert np.array_equal(b.array("reorderedRows"), rows)


def test_small_cluster_batches():
    """Several persistent launches (batch of 7 clusters) give the same permutation."""
    M, N, rp, ci = small_cases()["trefethen_small"]
    a = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE)
    b = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE, cluster_batch=7)
    assert a.stats()["num_clusters"] == b.stats()["num_clusters"]
    assert np.array_equal(a.array("reorderedRows"), b.array("reorderedRows"))


def _gpu_stats(plan):
    s = plan.stats()
    e = plan.evaluate()
    return {
        "numRowPanels": s["num_row_panels"], "numClusters": s["num_clusters"],
        "numDenseBlock": e["num_dense_block"], "averageDensity": e["average_density"],
        "originalNumDenseBlock": e["original_num_dense_block"],
        "originalAverageDensity": e["original_average_density"],
        "numDenseThreadBlocks": s["num_dense_thread_blocks"],
        "numSparseThreadBlocks": s["num_sparse_thread_blocks"],
        "numDenseData": e["num_dense_data"], "numSparseData": e["num_sparse_data"],
        "maxDense": s["max_dense_tiles_per_panel"],
        "rphmSparseTB": s["num_sparse_thread_blocks"],
    }


@pytest.mark.timeout(900)
@pytest.mark.parametrize("name", ["Trefethen_20000", "Trefethen_20000b", "mycielskian14",
                                  "mycielskian15", "mycielskian16"])
@pytest.mark.parametrize("alpha", ALPHAS)
def test_gpu_plan_matches_reference_logs(name, alpha):
    M, N, rp, ci = matrix(name)
    plan = Plan(M, N, rp, ci, alpha=alpha, delta=DELTAS[0], free_mem_bytes=REF_FREE_MEM)
    bad = {}
    for delta in DELTAS:
        plan.recolumn(delta)
        s = _gpu_stats(plan)
        for K in (32, 64, 128, 256):
            d = compare(expected_from_stats(s, K), record(name, alpha, delta, K))
            if d:
                bad[(delta, K)] = d
    assert not bad, bad


@functools.lru_cache(maxsize=None)
def nips_like_case():
    return synth.nips_like()


@pytest.mark.parametrize("name", ["ragged_empty_rows", "zipf", "wide_bs20", "blocky",
                                  "trefethen_small", "mycielskian10"])
@pytest.mark.parametrize("alpha", [0.1, 0.3, 0.9])
def test_cluster_filter_same_permutation(name, alpha):
    """The clustering's candidate filter (cluster_filter.hip: an MFMA bound of every pair's
    similarity, pairs that cannot reach alpha skipped by the chain) forced on: the permutation and
    cluster count equal the oracle's first-fit (rowReordering.cu:325-432, 893-1007), and the
    chain walks the same number of (position, cluster) pairs as without the filter."""
    M, N, rp, ci = small_cases()[name]
    on = Plan(M, N, rp, ci, alpha=alpha, delta=0.3, free_mem_bytes=FREE,
              tuning=tuning_from_env({"BSMR_CLUSTER_FILTER": "1"}))
    off = Plan(M, N, rp, ci, alpha=alpha, delta=0.3, free_mem_bytes=FREE,
               tuning=tuning_from_env({"BSMR_CLUSTER_FILTER": "0"}))
    s_on, s_off = on.stats(), off.stats()
    assert s_on["cluster_filter_used"] == 1 and s_off["cluster_filter_used"] == 0
    c = O.CSR.from_arrays(M, N, rp, ci)
    rows, ncl, _ = O.row_reorder(c, np.float32(alpha), O.block_size(M, N, FREE))
    assert s_on["num_clusters"] == ncl
    assert np.array_equal(on.array("reorderedRows"), rows)
    assert s_on["total_similarity_evals"] == s_off["total_similarity_evals"]
    assert s_on["exact_similarity_evals"] == s_off["exact_similarity_evals"]


@pytest.mark.parametrize("M,N,per_row,alpha", [(300, 400000, 100, 0.3), (600, 250000, 80, 0.1),
                                               (400, 180000, 150, 0.5)])
def test_cluster_filter_wide_tiles(M, N, per_row, alpha):
    """Wide patterns at the block-count ceiling of calculateBlockSize (~6,100 column blocks, so
    a clustering tile holds T = 6 representatives, as for reddit; the small cases above run
    T = 8): the filtered permutation equals the oracle's."""
    M, N, rp, ci = synth.random_rows(M, N, per_row, seed=M + N, zipf=1.05)
    gp = Plan(M, N, rp, ci, alpha=alpha, delta=0.3, free_mem_bytes=FREE,
              tuning=tuning_from_env({"BSMR_CLUSTER_FILTER": "1"}))
    st = gp.stats()
    assert st["cluster_filter_used"] == 1
    c = O.CSR.from_arrays(M, N, rp, ci)
    rows, ncl, _ = O.row_reorder(c, np.float32(alpha), O.block_size(M, N, FREE))
    assert st["num_clusters"] == ncl
    assert np.array_equal(gp.array("reorderedRows"), rows)


@pytest.mark.parametrize("scale,alpha", [(0.02, 0.3), (0.05, 0.3), (0.05, 0.1), (0.05, 0.7)])
def test_cluster_filter_reddit_like(scale, alpha):
    """A power-law graph (almost every position starts its own cluster, so the chain compares
    nearly all pairs): the filtered chain gives the same permutation as the unfiltered one."""
    M, N, rp, ci = synth.reddit_like(scale)
    perms, stats = [], []
    for f in ("1", "0"):
        plan = Plan(M, N, rp, ci, alpha=alpha, delta=0.3, free_mem_bytes=FREE,
                    tuning=tuning_from_env({"BSMR_CLUSTER_FILTER": f}))
        perms.append(plan.array("reorderedRows"))
        stats.append(plan.stats())
    assert stats[0]["cluster_filter_used"] == 1
    assert stats[0]["num_clusters"] == stats[1]["num_clusters"]
    assert np.array_equal(perms[0], perms[1])
    assert stats[0]["total_similarity_evals"] == stats[1]["total_similarity_evals"]


@pytest.mark.parametrize("batch", [0, 600])
def test_cluster_filter_auto_probe(batch):
    """The default policy (probe launch without the filter, then the filter) on a pattern above
    its row threshold, with the default and a small clusters-per-launch setting (the probe then
    shrinks to the launch's scratch): the permutation equals the unfiltered chain's."""
    M, N, rp, ci = synth.reddit_like(0.2)
    auto = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE, cluster_batch=batch)
    off = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE, cluster_batch=batch,
               tuning=tuning_from_env({"BSMR_CLUSTER_FILTER": "0"}))
    assert M >= 32768 and auto.stats()["cluster_filter_used"] == 1
    assert auto.stats()["num_clusters"] == off.stats()["num_clusters"]
    assert np.array_equal(auto.array("reorderedRows"), off.array("reorderedRows"))


def test_cluster_filter_nips_like_bit_exact():
    """nips-like (C1/C2's pattern) with the filter forced on: plan arrays equal the oracle's."""
    M, N, rp, ci = nips_like_case()
    gp = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE,
              tuning=tuning_from_env({"BSMR_CLUSTER_FILTER": "1"}))
    assert gp.stats()["cluster_filter_used"] == 1
    _, op, ncl = oracle_plan(M, N, rp, ci, 0.3, 0.3, FREE)
    assert gp.stats()["num_clusters"] == ncl
    assert_plans_equal(gp, op)


def test_nips_like_plan_bit_exact():
    M, N, rp, ci = nips_like_case()
    gp = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE)
    _, op, ncl = oracle_plan(M, N, rp, ci, 0.3, 0.3, FREE)
    assert gp.stats()["num_clusters"] == ncl
    assert_plans_equal(gp, op)


@pytest.mark.parametrize("layout", ["auto", "colmajor"])
@pytest.mark.parametrize("K", [16, 32, 48, 64, 96, 128, 256, 512])
@pytest.mark.parametrize("delta", [0.0, 0.3, 1.1])
def test_sddmm_values_checkdata(K, delta, layout):
    M, N, rp, ci = small_cases()["zipf"]
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=delta, free_mem_bytes=FREE, layout=layout)
    A = make_data(M * K)
    B = make_data(N * K)
    P = run_sddmm(plan, A, B, K, len(ci))
    c = O.CSR.from_arrays(M, N, rp, ci)
    ref = O.sddmm_cpu(c, K, A, B)
    assert np.isfinite(P).all()
    assert O.check_data(ref, P) == 0


@pytest.mark.parametrize("K,layout,lds_kb", [(32, "auto", 0), (64, "auto", 0), (128, "auto", 0),
                                             (128, "colmajor", 0), (128, "auto", 48),
                                             (256, "auto", 0), (512, "auto", 0),
                                             (512, "auto", 160)])
def test_sddmm_nips_like_checkdata(K, layout, lds_kb):
    M, N, rp, ci = nips_like_case()
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE, layout=layout,
                lds_budget_kb=lds_kb)
    A = make_data(M * K)
    B = make_data(N * K)
    P = run_sddmm(plan, A, B, K, len(ci))
    ref = O.sddmm_cpu(O.CSR.from_arrays(M, N, rp, ci), K, A, B)
    assert O.check_data(ref, P) == 0


@pytest.mark.parametrize("K,layout", [(128, "auto"), (128, "colmajor"), (128, "rowblock"),
                                      (64, "rowblock"), (256, "rowblock"), (512, "rowblock")])
def test_sddmm_blocky_dense_tiles(K, layout):
    M, N, rp, ci = small_cases()["blocky"]
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE, layout=layout)
    assert plan.stats()["num_dense_tiles"] > 0
    A = make_data(M * K)
    B = make_data(N * K)
    P = run_sddmm(plan, A, B, K, len(ci))
    ref = O.sddmm_cpu(O.CSR.from_arrays(M, N, rp, ci), K, A, B)
    assert O.check_data(ref, P) == 0


@pytest.mark.parametrize("world", [2, 3, 8])
def test_panel_shards_cover_every_output(world):
    M, N, rp, ci = nips_like_case()
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE)
    K = 64
    shards = [plan.shard(K, r, world) for r in range(world)]
    assert shards[0][0] == 0 and shards[-1][1] == plan.stats()["num_row_panels"]
    for (a0, a1), (b0, b1) in zip(shards, shards[1:]):
        assert a1 == b0 and a0 <= a1
    A = make_data(M * K)
    B = make_data(N * K)
    # the output buffer starts as NaN: every entry must be written exactly by its shard
    pieces = run_sddmm(plan, A, B, K, len(ci), panels=shards)
    assert np.isfinite(pieces).all()
    ref = O.sddmm_cpu(O.CSR.from_arrays(M, N, rp, ci), K, A, B)
    assert O.check_data(ref, pieces) == 0
    # a single shard leaves the other shards' outputs untouched
    p0, p1 = shards[world // 2]
    part = run_sddmm(plan, A, B, K, len(ci), panels=[(p0, p1)])
    rows = plan.array("reorderedRows")
    mine = np.zeros(len(ci), bool)
    for r in rows[p0 * 16: p1 * 16]:
        mine[rp[r]:rp[r + 1]] = True
    assert np.isfinite(part[mine]).all() and np.isnan(part[~mine]).all()


@pytest.mark.parametrize("K,dtype,world", [(128, 0, 4), (32, 0, 3), (256, 1, 5), (512, 2, 2),
                                           (128, 0, 1)])
def test_panel_shards_rowblock_kernel(K, dtype, world):
    """Row-panel shards on the row-block kernel (a layout per panel range) for fp32/fp16/bf16,
    and the column-major fallback (fp32 K=32): every output written once, by its own shard."""
    M, N, rp, ci = small_cases()["zipf"]
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE)
    shards = [plan.shard(K, r, world, dtype) for r in range(world)]
    A = make_data(M * K)
    B = make_data(N * K)
    P = run_sddmm(plan, A, B, K, len(ci), panels=shards, dtype=dtype)
    if dtype:
        A, B = half_values(A, dtype), half_values(B, dtype)
    ref = O.sddmm_cpu(O.CSR.from_arrays(M, N, rp, ci), K, A, B)
    assert np.isfinite(P).all()
    assert O.check_data(ref, P) == 0
    rows = plan.array("reorderedRows")
    for p0, p1 in shards:
        part = run_sddmm(plan, A, B, K, len(ci), panels=[(p0, p1)], dtype=dtype)
        mine = np.zeros(len(ci), bool)
        for r in rows[p0 * 16: p1 * 16]:
            mine[rp[r]:rp[r + 1]] = True
        assert np.isfinite(part[mine]).all() and np.isnan(part[~mine]).all(), (p0, p1)
        assert O.check_data(ref[mine], part[mine]) == 0


@pytest.mark.parametrize("env,K,dtype", [
    ({"BSMR_TILE_MIN_F32": "0"}, 128, 0),      # every fp32 tile on MFMA
    ({"BSMR_TILE_MIN_F32": "100"}, 128, 0),    # some tiles demoted to residual entries
    ({"BSMR_TILE_MIN_F32": "257"}, 64, 0),     # none kept (default)
    ({"BSMR_TILE_MIN_HALF": "0"}, 256, 1),
    ({"BSMR_TILE_MIN_HALF": "200"}, 256, 2),
    ({"BSMR_TILE_MIN_HALF": "257"}, 512, 2),
    ({"BSMR_L2_RANGE_KB": "64"}, 128, 0),      # m > 1 column ranges per XCD, several rounds
    ({"BSMR_L2_RANGE_KB": "64", "BSMR_TILE_MIN_F32": "0"}, 64, 0),
    ({"BSMR_L2_RANGE_KB": "64"}, 256, 1),
    ({"BSMR_PIECE_WEIGHT": "0"}, 128, 0),     # item cut by entries + tiles only
    ({"BSMR_PIECE_WEIGHT": "16"}, 256, 1),    # pieces dominate the item cost
    ({"BSMR_SHARD_PIECE_WEIGHT": "1"}, 128, 0),   # shard cuts (checked below) by entries mostly
    ({"BSMR_SHARD_PIECE_WEIGHT": "16"}, 64, 2),
    ({"BSMR_TILE_MIN_F32": "0"}, 32, 0),       # 128-byte rows, fp32 tiles on MFMA
    ({}, 32, 0),                               # 128-byte rows (8 rows per staged KiB)
    ({"BSMR_TILE_MIN_HALF": "0"}, 64, 1),      # 128-byte rows, half tiles on MFMA
    ({}, 64, 2),
    ({"BSMR_ORIG_ROWS": "1"}, 128, 0),         # original-order row blocks, every entry residual
    ({"BSMR_ORIG_ROWS": "1"}, 256, 1),
    ({"BSMR_ORIG_ROWS": "1"}, 32, 0),
    ({"BSMR_ORIG_ROWS": "1", "BSMR_L2_RANGE_KB": "64"}, 128, 0),
    # results staged in LDS, written per item in CSR order (auto for P > 8 MiB)
    ({"BSMR_OUT_STAGED": "1"}, 128, 0),
    ({"BSMR_OUT_STAGED": "1"}, 32, 0),
    ({"BSMR_OUT_STAGED": "1"}, 256, 1),
    ({"BSMR_OUT_STAGED": "1", "BSMR_TILE_MIN_HALF": "0"}, 512, 2),
    ({"BSMR_OUT_STAGED": "1", "BSMR_ORIG_ROWS": "1"}, 128, 0),
    ({"BSMR_OUT_STAGED": "1", "BSMR_L2_RANGE_KB": "64", "BSMR_TILE_MIN_F32": "0"}, 64, 0),
    # item scheduling: the round-2 layout, fixed caps, and one with staged output
    ({"BSMR_ITEM_SCHED": "0", "BSMR_ITEM_CAP": "0"}, 128, 0),
    ({"BSMR_ITEM_CAP": "1"}, 128, 0),
    ({"BSMR_ITEM_CAP": "1.25", "BSMR_OUT_STAGED": "1"}, 256, 1),
    ({"BSMR_ITEM_SCHED": "0"}, 512, 2),
    ({"BSMR_LATE_B": "0"}, 128, 0),
    ({"BSMR_RB_ROWS": "16"}, 128, 0),
    ({"BSMR_RB_ROWS": "48", "BSMR_OUT_STAGED": "1"}, 512, 0),
])
def test_rowblock_layout_variants(env, K, dtype):
    """Launch-layout switches (tile demotion thresholds, L2 column ranges, piece order) on the
    blocky pattern (dense tiles and residual entries) and a zipf pattern: values unchanged."""
    tun = tuning_from_env(env)  # the knobs by their BSMR_* names (bsmr_tuning_from_env)
    for name in ("blocky", "wide_bs20"):
        M, N, rp, ci = small_cases()[name]
        plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE, layout="rowblock",
                    tuning=tun)
        A = make_data(M * K)
        B = make_data(N * K)
        P = run_sddmm(plan, A, B, K, len(ci), dtype=dtype)
        if dtype:
            A, B = half_values(A, dtype), half_values(B, dtype)
        ref = O.sddmm_cpu(O.CSR.from_arrays(M, N, rp, ci), K, A, B)
        assert np.isfinite(P).all(), name
        assert O.check_data(ref, P) == 0, name
        # shards of the same plan agree
        shards = [plan.shard(K, r, 3, dtype) for r in range(3)]
        Ps = run_sddmm(plan, A, B, K, len(ci), panels=shards, dtype=dtype)
        assert np.isfinite(Ps).all() and O.check_data(ref, Ps) == 0, name


@functools.lru_cache(maxsize=None)
def wide_case():
    # N = 400 K: 512-byte B rows make 25.6 MB per XCD share, so the staged default of 8 MiB
    # column ranges gives m = 4 ranges per XCD (the 4 MiB rule gave 7), with split row blocks
    return synth.random_rows(2048, 400000, 400, seed=9, zipf=1.1)


@pytest.mark.parametrize("env,K,dtype", [
    ({"BSMR_OUT_STAGED": "1"}, 128, 0),                            # C4's default: 8 MiB ranges
    ({"BSMR_OUT_STAGED": "1"}, 256, 1),                            # C3's row size, fp16
    ({"BSMR_OUT_STAGED": "1", "BSMR_L2_RANGE_KB": "8192"}, 128, 0),  # the same, set explicitly
    ({"BSMR_OUT_STAGED": "1", "BSMR_L2_RANGE_KB": "4096"}, 128, 0),  # the round-3 staged rule
    ({}, 128, 0),                                                  # unstaged (P < 8 MiB)
    ({"BSMR_OUT_STAGED": "1", "BSMR_L2_RANGE_KB": "512"}, 256, 2),  # small ranges in bf16
])
def test_staged_default_column_ranges_wide(env, K, dtype):
    """The staged 512-byte-row default (8 MiB XCD column ranges, plan.hip build_rowblock_layout)
    on a pattern wide enough for several ranges per XCD: values equal the oracle's, and the
    whole-plan launch splits row blocks by range (more items than row blocks)."""
    M, N, rp, ci = wide_case()
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE, layout="rowblock",
                tuning=tuning_from_env(env))
    A = make_data(M * K)
    B = make_data(N * K)
    P = run_sddmm(plan, A, B, K, len(ci), dtype=dtype)
    if dtype:
        A, B = half_values(A, dtype), half_values(B, dtype)
    ref = O.sddmm_cpu(O.CSR.from_arrays(M, N, rp, ci), K, A, B)
    assert np.isfinite(P).all()
    assert O.check_data(ref, P) == 0
    s = plan.stats()  # 512-byte rows: layout slot 2 (fp32 K = 128, half K = 256)
    rb = s["rb_rows"][2]
    assert rb > 0 and s["rb_items"][2] > (s["num_reordered_rows"] + rb - 1) // rb
    shards = [plan.shard(K, r, 2, dtype) for r in range(2)]
    Ps = run_sddmm(plan, A, B, K, len(ci), panels=shards, dtype=dtype)
    assert np.isfinite(Ps).all() and O.check_data(ref, Ps) == 0


def test_values_independent_of_layout_permutation():
    """Size-independent property: P of the same S is identical for every alpha/delta plan."""
    M, N, rp, ci = small_cases()["zipf"]
    K = 64
    A = make_data(M * K)
    B = make_data(N * K)
    ref = O.sddmm_cpu(O.CSR.from_arrays(M, N, rp, ci), K, A, B)
    for alpha, delta in [(0.1, 0.0), (0.5, 0.1), (0.9, 0.9)]:
        plan = Plan(M, N, rp, ci, alpha=alpha, delta=delta, free_mem_bytes=FREE)
        P = run_sddmm(plan, A, B, K, len(ci))
        assert O.check_data(ref, P) == 0


@pytest.mark.parametrize("case,K,layout,nb", [("zipf", 128, "auto", 3), ("zipf", 64, "colmajor", 2),
                                               ("zipf", 96, "auto", 4), ("banded", 128, "auto", 2)])
def test_sddmm_batch_each_batch_checkdata(case, K, layout, nb):
    """sddmm_gpu_batch semantics: batch b = (A_b, B_b) at strides M*K / N*K, P_b at b*nnz
    (banded: the original-order row-block layout)."""
    torch = torch_cuda()
    if case == "banded":
        M, N, rp, ci = synth.banded_fem_like(3000, 22, seed=6, band=48)
    else:
        M, N, rp, ci = small_cases()[case]
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE, layout=layout)
    A = make_data(nb * M * K)
    B = make_data(nb * N * K)[::-1].copy()  # different values per batch
    dA = torch.from_numpy(A).cuda()
    dB = torch.from_numpy(B).cuda()
    nnz = len(ci)
    dP = torch.full((nb * nnz,), float("nan"), dtype=torch.float32, device="cuda")
    plan.sddmm_batch(nb, dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(),
                     stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    P = dP.cpu().numpy()
    c = O.CSR.from_arrays(M, N, rp, ci)
    for b in range(nb):
        ref = O.sddmm_cpu(c, K, A[b * M * K:(b + 1) * M * K], B[b * N * K:(b + 1) * N * K])
        assert O.check_data(ref, P[b * nnz:(b + 1) * nnz]) == 0, b


@pytest.mark.parametrize("K,dtype,chosen", [(128, 0, True), (256, 1, True), (64, 2, None)])
def test_original_order_row_blocks_banded(K, dtype, chosen):
    """Banded FEM-like pattern with random couplings (the C3 shape, small): the reordering
    scatters the band, so the whole-plan launch picks original-order row blocks (sparse-row
    rule, cost model); values match the oracle, and shards (reordered panel layouts) agree."""
    M, N, rp, ci = synth.banded_fem_like(6000, 22, seed=5, band=48)
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE, layout="rowblock")
    A = make_data(M * K)
    B = make_data(N * K)
    P = run_sddmm(plan, A, B, K, len(ci), dtype=dtype)
    if dtype:
        A, B = half_values(A, dtype), half_values(B, dtype)
    ref = O.sddmm_cpu(O.CSR.from_arrays(M, N, rp, ci), K, A, B)
    assert np.isfinite(P).all() and O.check_data(ref, P) == 0
    if chosen:  # (1024-row blocks of 128-byte rows: the rule may keep the reordered layout)
        slot = {128: 0, 256: 1, 512: 2}[K * (4 if dtype == 0 else 2)]
        assert plan.stats()["rb_orig_rows"] == 1 << slot  # the original-order layout was chosen
    shards = [plan.shard(K, r, 2, dtype) for r in range(2)]
    Ps = run_sddmm(plan, A, B, K, len(ci), panels=shards, dtype=dtype)
    assert np.isfinite(Ps).all() and O.check_data(ref, Ps) == 0
