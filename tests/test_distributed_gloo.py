"""Multi-process (world_size 2, gloo, CPU) tests of the row-panel split bench.py runs on GPUs
(bsmr/dist.py): the row stage is computed once on rank 0 and broadcast, both ranks
derive the same panel cuts from the same plan, each rank computes only its panels' outputs from
its own A rows (shard_a_rows), and P is assembled bit-exactly on rank 0 (each rank's outputs
compacted in plan order and scattered back, gather_compact; or its contiguous CSR segment,
gather_segments). World 8: the row-block cost cut, its measured-time re-cut and the assembly with
uneven and empty shards, bit for bit (-0.0 included) against a single-rank run. The per-shard
compute is the CPU here (no device); the GPU path is tests/test_gpu_shards.py."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "sddmm-gpu_amd"), os.path.join(root, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    import torch

    import bsmr
    import oracle_lib as O
    from bsmr import dist as D
    from bsmr import synth

    r, w = D.init("gloo")
    assert (r, w) == (rank, world)
    res = {"rank": rank}
    # B broadcast: rank 0 holds the makeData stream, the others receive it
    n = 4096
    B = torch.from_numpy(bsmr.make_data(n)) if rank == 0 else torch.zeros(n)
    D.broadcast_(B, 0)
    res["b_ok"] = bool(np.array_equal(B.numpy(), bsmr.make_data(n)))
    res["t"] = D.max_over_ranks(1.5 + rank, "cpu")
    res["all"] = D.all_values(10 + rank, "cpu")

    # the weak-scaling workload: 2 stacked copies of a small pattern
    M0, N, rp0, ci0 = synth.random_rows(300, 2000, 30, seed=41, zipf=1.1, empty_frac=0.05)
    M, N, rp, ci = synth.stack_copies(M0, N, rp0, ci0, world)
    c = O.CSR.from_arrays(M, N, rp, ci)
    alpha, delta, K = np.float32(0.3), np.float32(0.3), 64
    bs = O.block_size(M, N, 288 * 1024 ** 3)
    # row stage: clustered on rank 0 only, shipped as (header, rows)
    hdr, rows = None, None
    if rank == 0:
        rows, ncl, _ = O.row_reorder(c, alpha, bs)
        hdr = bsmr.RowStage(M=M, N=N, nnz=len(ci), block_size=bs,
                            num_zero_rows=M - len(rows), num_reordered_rows=len(rows),
                            num_clusters=ncl, alpha=alpha)
    hdr, rows_t = D.broadcast_row_stage(hdr, rows, "cpu")
    rows = rows_t.numpy().view(np.uint32)[:hdr.num_reordered_rows].copy()
    ref_rows, ref_ncl, _ = O.row_reorder(c, alpha, bs)
    res["rows_ok"] = bool(np.array_equal(rows, ref_rows)) and hdr.num_clusters == ref_ncl
    # the same plan on both ranks -> the same cuts
    plan = O.Plan(c, rows, hdr.num_clusters, delta)
    cuts = bsmr.shard_cuts(plan.array("blockOffsets"), plan.array("sparseValueOffsets"), K, world)
    p0, p1 = D.panel_range(cuts, rank)
    res["cut"] = (p0, p1)
    # this rank's outputs from its own A rows only
    A = bsmr.make_data(M * K)
    Bf = bsmr.make_data(N * K)
    A_local = D.shard_a_rows(A, K, rows, p0, p1)
    P = np.zeros(len(ci), np.float32)
    for j, row in enumerate(rows[16 * p0:min(16 * p1, len(rows))]):
        for e in range(rp[row], rp[row + 1]):
            P[e] = np.dot(A_local[j].astype(np.float64), Bf[ci[e] * K:(ci[e] + 1) * K])
    pos_all = [D.shard_positions(rp, rows, *D.panel_range(cuts, r)) for r in range(world)]
    Pg = D.gather_compact(torch.from_numpy(P), pos_all[rank], [len(x) for x in pos_all], len(ci),
                          pos_all if rank == 0 else None, 0)
    if rank == 0:
        ref = O.sddmm_cpu(c, K, A, Bf)
        res["p_errors"] = O.check_data(ref, Pg)
        res["p_written"] = int(np.count_nonzero(Pg))
        res["nnz"] = len(ci)
    # the local split (bench.py --shard local, the C2 weak-scaling default): contiguous original
    # row panels of equal stored entries (= the stacked copies), each rank's outputs written at
    # their contiguous CSR positions
    q0, q1 = D.row_range_cut(rp, rank, world)
    res["local_cut"] = (q0, q1)
    P2 = np.zeros(len(ci), np.float32)
    A_rows = np.asarray(A).reshape(-1, K)[q0:q1]  # only this rank's rows of A
    for j, row in enumerate(range(q0, q1)):
        for e in range(rp[row], rp[row + 1]):
            P2[e] = np.dot(A_rows[j].astype(np.float64), Bf[ci[e] * K:(ci[e] + 1) * K])
    e0, e1 = int(rp[q0]), int(rp[q1])
    Pg2 = D.gather_segments(torch.from_numpy(P2[e0:e1].copy()), e0, e1, len(ci), 0)
    if rank == 0:
        res["p2_errors"] = O.check_data(ref, Pg2)
        res["p2_written"] = int(np.count_nonzero(Pg2))
    # the segments gathered as they are (bench.py's local split): bit-exact, including the sign of
    # a zero output
    seg = P2[e0:e1].copy()
    seg[0] = -0.0
    Pg3 = D.gather_segments(torch.from_numpy(seg), e0, e1, len(ci), 0)
    Pall = D.gather_segments(torch.from_numpy(P2[e0:e1].copy()), e0, e1, len(ci), 0)
    if rank == 0:
        res["seg_equal"] = bool(np.array_equal(Pall.view(np.uint32), Pg2.view(np.uint32)))
        res["seg_negzero"] = [bool(np.signbit(Pg3[int(rp[q])]) and Pg3[int(rp[q])] == 0)
                              for q in (0, 300)]
    import torch.distributed as dist
    dist.destroy_process_group()
    q.put(res)


@pytest.mark.timeout(300)
def test_gloo_world2_row_stage_shards_and_p_gather():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in procs), key=lambda d: d["rank"])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    r0, r1 = res
    assert r0["b_ok"] and r1["b_ok"]
    assert r0["t"] == r1["t"] == 2.5
    assert r0["all"] == r1["all"] == [10.0, 11.0]
    assert r0["rows_ok"] and r1["rows_ok"]
    (a0, a1), (b0, b1) = r0["cut"], r1["cut"]
    assert a0 == 0 and a1 == b0 and a0 < a1 < b1
    assert r0["p_errors"] == 0 and r0["p_written"] == r0["nnz"]
    assert r0["local_cut"] == (0, 300) and r1["local_cut"] == (300, 600)  # the two copies
    assert r0["p2_errors"] == 0 and r0["p2_written"] == r0["nnz"]
    assert r0["seg_equal"] and r0["seg_negzero"] == [True, True]


def test_row_range_cut():
    """Contiguous row panels of (nearly) equal stored entries, exact at equal-block boundaries,
    covering every row once, including empty rows and more ranks than non-empty rows."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "sddmm-gpu_amd"))
    from bsmr import dist as D
    rp = np.array([0, 5, 10, 15, 20], dtype=np.uint32)  # 4 rows of 5
    assert [D.row_range_cut(rp, r, 2) for r in range(2)] == [(0, 2), (2, 4)]
    assert [D.row_range_cut(rp, r, 4) for r in range(4)] == [(0, 1), (1, 2), (2, 3), (3, 4)]
    rp = np.array([0, 0, 12, 12, 13, 20, 20], dtype=np.uint32)  # empty and uneven rows
    for world in (1, 2, 3, 5, 8):
        cuts = [D.row_range_cut(rp, r, world) for r in range(world)]
        assert cuts[0][0] == 0 and cuts[-1][1] == 6
        assert all(a[1] == b[0] for a, b in zip(cuts, cuts[1:]))
        assert all(a <= b for a, b in cuts)


def _worker8(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "sddmm-gpu_amd"), os.path.join(root, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    import torch

    import bsmr
    import oracle_lib as O
    from bsmr import dist as D
    from bsmr import synth

    D.init("gloo")
    res = {"rank": rank}
    # 200 rows -> 13 panels -> 7 row blocks of 2 panels (the last one short) for 8 ranks: at least
    # one shard is empty, the others uneven
    M, N, rp, ci = synth.random_rows(200, 700, 25, seed=43, zipf=1.2, empty_frac=0.03)
    c = O.CSR.from_arrays(M, N, rp, ci)
    rows, ncl, _ = O.row_reorder(c, np.float32(0.3), O.block_size(M, N, 288 * 1024 ** 3))
    plan = O.Plan(c, rows, ncl, np.float32(0.3))
    bo, so = plan.array("blockOffsets"), plan.array("sparseValueOffsets")
    P = len(bo) - 1
    ppr = 2
    nblk = (P + ppr - 1) // ppr
    # block cost: its stored entries + 16 per dense tile (any positive model will do: every rank
    # derives the same cuts from the same plan)
    cost = [float(so[min(P, ppr * (b + 1))] - so[ppr * b]) + 16.0 * float(bo[min(P, ppr * (b + 1))] - bo[ppr * b]) + 1.0
            for b in range(nblk)]
    cuts = bsmr.cost_cuts(cost, ppr, P, world)
    res["model_cuts"] = cuts
    # measured shard times: the model cost of the shard times a rank-dependent speed (a slow
    # device), gathered over the ranks, then every rank re-cuts from the same numbers
    speed = 1.0 + 0.5 * (rank % 3)
    p0, p1 = D.panel_range(cuts, rank)
    mine = sum(cost[b] for b in range(p0 // ppr, (p1 + ppr - 1) // ppr)) if p1 > p0 else 0.0
    ms = D.all_values(mine * speed * 1e-3, "cpu")
    cuts2 = bsmr.cost_cuts(cost, ppr, P, world, prev_cuts=cuts, shard_ms=ms)
    res["rebalanced_cuts"] = cuts2
    p0, p1 = D.panel_range(cuts2, rank)
    res["cut"] = (p0, p1)
    # this rank's outputs from its own A rows only; every 97th output forced to -0.0 (a computed
    # value whose sign the assembly must keep)
    K = 32
    A = bsmr.make_data(M * K).reshape(M, K)
    Bf = bsmr.make_data(N * K).reshape(N, K)[::-1].copy()

    def outputs(q0, q1):
        out = np.zeros(len(ci), np.float32)
        for row in rows[16 * q0:min(16 * q1, len(rows))]:
            for e in range(rp[row], rp[row + 1]):
                out[e] = np.float32(-0.0) if e % 97 == 0 else np.dot(A[row], Bf[ci[e]])
        return out

    dP = torch.from_numpy(outputs(p0, p1))
    pos_all = [D.shard_positions(rp, rows, cuts2[r], cuts2[r + 1]) for r in range(world)]
    counts = [len(x) for x in pos_all]
    res["counts"] = counts
    Pg = D.gather_compact(dP, pos_all[rank], counts, len(ci), pos_all if rank == 0 else None, 0)
    if rank == 0:
        whole = outputs(0, P)  # the single-rank run: every panel on one rank
        res["bitexact"] = bool(np.array_equal(Pg.view(np.uint32), whole.view(np.uint32)))
        res["negzero"] = int(np.count_nonzero(np.signbit(Pg) & (Pg == 0)))
        res["nnz"] = len(ci)
        res["P"] = P
    import torch.distributed as dist
    dist.destroy_process_group()
    q.put(res)


@pytest.mark.timeout(300)
def test_gloo_world8_cut_rebalance_and_exact_assembly():
    """World 8 on gloo: the row-block cost cut (bsmr_cost_cuts, the host form of
    bsmr_plan_shard_dtype), its measured-time re-cut (bsmr_plan_shard_rebalance's rule) from
    gathered per-rank times, identical on every rank, and the bit-exact assembly of P from shards
    that are uneven and include an empty one (gather_compact: plan-order compaction, rank 0
    scatters back), compared bit for bit, -0.0 included, with a single-rank run."""
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker8, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=280) for _ in procs), key=lambda d: d["rank"])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    r0 = res[0]
    for r in res:  # the same cuts on every rank, before and after the re-cut
        assert r["model_cuts"] == r0["model_cuts"] and r["rebalanced_cuts"] == r0["rebalanced_cuts"]
        assert r["counts"] == r0["counts"]
    cuts = r0["rebalanced_cuts"]
    assert cuts[0] == 0 and cuts[-1] == r0["P"] and all(a <= b for a, b in zip(cuts, cuts[1:]))
    assert r0["model_cuts"] != cuts  # the slow ranks' shards moved
    assert any(c == 0 for c in r0["counts"]), "no empty shard"
    assert len(set(r0["counts"])) > 2, "shards not uneven"
    assert sum(r0["counts"]) == r0["nnz"]
    assert r0["bitexact"] and r0["negzero"] > 0
