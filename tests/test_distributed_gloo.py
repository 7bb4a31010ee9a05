"""Multi-process (world_size 2, gloo, CPU) tests of the sharded-run plumbing used by bench.py:
B broadcast from rank 0, slowest-rank timing, and a disjoint cover of the row panels by the
cost-model shard cuts. The GPU data path itself has no collective."""
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
    sys.path.insert(0, os.path.join(root, "sddmm-gpu_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    import torch

    import bsmr
    from bsmr import dist as D

    r, w = D.init("gloo")
    assert (r, w) == (rank, world)
    # B broadcast: rank 0 holds the makeData stream, the others receive it
    n = 4096
    B = torch.from_numpy(bsmr.make_data(n)) if rank == 0 else torch.zeros(n)
    D.broadcast_(B, 0)
    ok_b = bool(np.array_equal(B.numpy(), bsmr.make_data(n)))
    t = D.max_over_ranks(1.5 + rank, "cpu")
    # every rank computes the same cuts from the same plan offsets; ranges tile [0, P)
    bo = np.cumsum([0] + [3, 0, 5, 1, 7, 2, 2, 9, 0, 4]).astype(np.uint32)
    so = np.cumsum([0] + [100, 40, 0, 900, 10, 10, 300, 0, 5, 77]).astype(np.uint32)
    cuts = bsmr.shard_cuts(bo, so, 128, w)
    p0, p1 = D.panel_range(cuts, rank)
    total = D.sum_over_ranks(p1 - p0, "cpu")
    import torch.distributed as dist
    dist.destroy_process_group()
    q.put((rank, ok_b, t, p0, p1, total))


@pytest.mark.timeout(300)
def test_gloo_world2_broadcast_timing_and_shards():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, b0, t0, a0, a1, tot0), (r1, b1, t1, c0, c1, tot1) = res
    assert b0 and b1
    assert t0 == t1 == 2.5
    assert a0 == 0 and a1 == c0 and c1 == 10 and tot0 == tot1 == 10
