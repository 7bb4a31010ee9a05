"""Row-panel sharded SDDMM over several GPUs: one process per GPU over
torch.distributed (backend "nccl" = RCCL over xGMI on MI355X; "gloo" for CPU tests and 1-GPU
rehearsals).

The reference has no multi-GPU code (its launcher is single-GPU, sddmmKernel.cu:2540-2663). The
split built here:

1. **Global plan, clustered once.** A bit-exact permutation needs the global first-fit over all
   rows, so rank 0 builds the plan (``bsmr_plan_create``) and broadcasts its row stage (the
   ``bsmr_row_stage`` header and the reordered rows, u32 on the device) over RCCL. The other
   ranks rebuild the column stage from it (``bsmr_plan_import_rows``): clustering is most of the
   plan time (reddit_like x1 on MI355X: 11.0 s of a 13 s plan), the column stage
   a deterministic O(nnz) pass (0.18 s) that is cheaper to recompute than to ship (its arrays are
   ~12 B per entry, ~2.8 GB for reddit_like x1, against 0.9 MB of row stage).
2. **Panel cut.** Every rank holds the same global plan, so every rank computes the same cost-model
   cuts (``bsmr_plan_shard_dtype``) without talking: contiguous panel ranges [p0, p1).
3. **A partitioned.** A rank uploads only the A rows of its panels, in reordered order
   (``shard_a_rows``), and runs ``bsmr_sddmm_panels_local`` on them.
4. **B broadcast once** from rank 0 (RCCL), outside the timed region.
5. **P gathered** to rank 0, bit-exact and 1/N of the entries per rank: the local split gathers
   each rank's contiguous CSR segment (``gather_segments``); a shard of the global plan owns
   scattered rows, so it sends its outputs compacted in plan order (its reordered rows in turn,
   each row's CSR segment) and rank 0 scatters them through the positions it derives from the
   same plan (``shard_positions``, ``gather_compact``) — no arithmetic, so -0.0 stays -0.0.

The timed loop has no collective; the whole-job time is the slowest rank's.
"""
import os
import time

import numpy as np


def env_rank_world():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend):
    """Initialise the default process group from the torchrun environment (MASTER_ADDR/PORT)."""
    import torch.distributed as dist

    if not dist.is_initialized():
        dist.init_process_group(backend)
    return dist.get_rank(), dist.get_world_size()


def _backend():
    import torch.distributed as dist

    return dist.get_backend()


def _comm(t):
    """The tensor the collective runs on: gloo has no reduce for device tensors, so it gets a
    host copy; RCCL takes the device tensor as is."""
    return t.cpu() if _backend() == "gloo" and t.is_cuda else t


def broadcast_(tensor, src=0):
    """In-place broadcast (e.g. B, generated on rank 0 and sent once before timing)."""
    import torch.distributed as dist

    c = _comm(tensor)
    dist.broadcast(c, src=src)
    if c is not tensor:
        tensor.copy_(c)
    return tensor


def max_over_ranks(value, device):
    """Max of a float over ranks (whole-job time = slowest rank)."""
    import torch
    import torch.distributed as dist

    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    c = _comm(t)
    dist.all_reduce(c, op=dist.ReduceOp.MAX)
    return float(c.item())


def sum_over_ranks(value, device):
    import torch
    import torch.distributed as dist

    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    c = _comm(t)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(c.item())


def all_values(value, device):
    """Every rank's float, in rank order (per-rank times and counts for the report)."""
    import torch
    import torch.distributed as dist

    w = dist.get_world_size()
    t = torch.zeros(w, dtype=torch.float64, device=device)
    t[dist.get_rank()] = float(value)
    c = _comm(t)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return [float(x) for x in c.cpu().tolist()]


def panel_range(cuts, rank):
    """Row panels [p0, p1) of `rank` from cost-model cut points (bsmr.shard_cuts)."""
    cuts = np.asarray(cuts)
    return int(cuts[rank]), int(cuts[rank + 1])


def broadcast_row_stage(hdr, rows, device):
    """Ship a row stage from rank 0: `hdr` (RowStage) and `rows` (a uint32 numpy array, or a
    callable that fills the int32 tensor to be sent, e.g. a device-to-device export) on rank 0,
    anything elsewhere. Returns (hdr, rows tensor int32 on `device`) on every rank.

    The header travels as its bytes, the rows as one device buffer (RCCL reads it in place)."""
    import torch
    import torch.distributed as dist

    from . import RowStage

    rank = dist.get_rank()
    hdr_bytes = torch.zeros(len(bytes(RowStage())), dtype=torch.uint8, device=device)
    if rank == 0:
        hdr_bytes.copy_(torch.from_numpy(hdr.to_array()))
    broadcast_(hdr_bytes, 0)
    hdr = RowStage.from_array(hdr_bytes.cpu().numpy())
    out = torch.empty(max(hdr.num_reordered_rows, 1), dtype=torch.int32, device=device)
    if rank == 0:
        if callable(rows):
            rows(out)
        else:
            out[:hdr.num_reordered_rows].copy_(
                torch.from_numpy(np.ascontiguousarray(rows, np.uint32).view(np.int32)))
    broadcast_(out, 0)
    return hdr, out


def distribute_plan(M, N, rowptr, colidx, device, alpha=0.3, delta=0.3, layout="auto",
                    free_mem_bytes=0):
    """The global plan on every rank, clustered once (rank 0) and shipped as its row stage.

    Returns (plan, info): info["plan_build_s"] is rank 0's full plan build, info["distribute_ms"]
    the row-stage broadcast plus the local column stage (bsmr_plan_import_rows) on this rank.
    """
    import torch
    import torch.distributed as dist

    from . import Plan

    rank = dist.get_rank()
    dev = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
    info = {"plan_build_s": 0.0}
    plan, hdr = None, None
    if rank == 0:
        t0 = time.perf_counter()
        plan = Plan(M, N, rowptr, colidx, alpha=alpha, delta=delta, device=dev.index,
                    layout=layout, free_mem_bytes=free_mem_bytes)
        info["plan_build_s"] = time.perf_counter() - t0
        hdr, _ = plan.export_rows()
    dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    # rank 0 writes the rows straight into the device buffer the broadcast sends
    hdr, rows = broadcast_row_stage(hdr, lambda t: plan.export_rows(t.data_ptr()), dev)
    torch.cuda.synchronize(dev)
    info["row_stage_bcast_ms"] = (time.perf_counter() - t0) * 1e3
    info["row_stage_bytes"] = int(len(bytes(hdr)) + 4 * hdr.num_reordered_rows)
    if rank != 0:
        plan = Plan.from_row_stage(rowptr, colidx, hdr, rows.data_ptr(), delta=delta,
                                   device=dev.index, layout=layout)
    torch.cuda.synchronize(dev)
    info["distribute_ms"] = (time.perf_counter() - t0) * 1e3
    return plan, info


def row_range_cut(rowptr, rank, world):
    """Original rows [r0, r1) of `rank` when S is cut into `world` contiguous row panels of
    (nearly) equal stored entries (the cut is the first row whose CSR offset reaches each
    target, so equal blocks such as stacked copies split exactly at their boundaries)."""
    rp = np.asarray(rowptr, dtype=np.int64)
    M, nnz = len(rp) - 1, int(rp[-1])
    cuts = [0] + [min(M, int(np.searchsorted(rp, nnz * r // world, side="left")))
                  for r in range(1, world)] + [M]
    for r in range(1, world + 1):
        cuts[r] = max(cuts[r], cuts[r - 1])
    return cuts[rank], cuts[rank + 1]


def shard_a_rows(A, K, reordered_rows, p0, p1):
    """The A rows of reordered positions [16 p0, min(16 p1, R)) in that order (host, row-major):
    the dA_local of bsmr_sddmm_panels_local."""
    A = np.asarray(A).reshape(-1, K)
    q1 = min(16 * p1, len(reordered_rows))
    return np.ascontiguousarray(A[np.asarray(reordered_rows[16 * p0:q1], dtype=np.int64)])


def shard_positions(rowptr, reordered_rows, p0, p1):
    """CSR positions of the outputs of panels [p0, p1) of a plan, in plan order: the reordered
    rows 16 p0 .. min(16 p1, R) - 1 in turn, each row's CSR segment [rowptr[r], rowptr[r + 1])
    (int64). Every rank derives every rank's list from the plan it holds; nothing is sent."""
    rp = np.asarray(rowptr, dtype=np.int64)
    rows = np.asarray(reordered_rows[16 * p0:min(16 * p1, len(reordered_rows))], dtype=np.int64)
    starts = rp[rows]
    lens = rp[rows + 1] - starts
    total = int(lens.sum())
    if total == 0:
        return np.zeros(0, np.int64)
    # position j of the list = starts[row of j] + (j - first list index of that row)
    first = np.cumsum(lens) - lens
    return np.repeat(starts - first, lens) + np.arange(total, dtype=np.int64)


def gather_compact(dP, positions, counts, nnz, all_positions=None, dst=0):
    """P in CSR order on rank `dst` from row-panel shards of one global plan. This rank wrote its
    outputs into dP (nnz long; positions = its shard_positions list); it sends them compacted in
    that order, padded to the longest shard (counts = every rank's list length, the same on every
    rank). On dst, all_positions[r] is rank r's list: the values are scattered back through it.
    Bit-exact (no arithmetic, -0.0 included); each rank sends its own entries only. Returns the
    host array on dst, None elsewhere."""
    import torch
    import torch.distributed as dist

    w, rank = dist.get_world_size(), dist.get_rank()
    width = max(max(int(c) for c in counts), 1)
    send = torch.zeros(width, dtype=torch.float32, device=dP.device)
    n = int(counts[rank])
    if n:
        idx = torch.from_numpy(np.ascontiguousarray(positions, np.int64)).to(dP.device)
        send[:n] = dP.index_select(0, idx)
    send = _comm(send)
    bufs = [torch.empty_like(send) for _ in range(w)] if rank == dst else None
    dist.gather(send, bufs, dst=dst)
    if rank != dst:
        return None
    P = np.zeros(int(nnz), np.float32)
    for r in range(w):
        k = int(counts[r])
        if k:
            P[np.asarray(all_positions[r], np.int64)] = bufs[r][:k].cpu().numpy()
    return P


def gather_segments(dP_seg, e0, e1, nnz, dst=0):
    """P in CSR order on rank `dst` from each rank's contiguous CSR segment [e0, e1) (the local
    split: a rank's rows are one range of original rows). Bit-exact (no arithmetic), and each
    rank sends only its segment (padded to the longest). Returns the host array on dst."""
    import torch
    import torch.distributed as dist

    w, rank = dist.get_world_size(), dist.get_rank()
    dev = dP_seg.device
    bounds = torch.zeros(2 * w, dtype=torch.int64, device=dev)
    bounds[2 * rank], bounds[2 * rank + 1] = int(e0), int(e1)
    c = _comm(bounds)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    b = [int(x) for x in c.cpu().tolist()]
    width = max(max(b[2 * r + 1] - b[2 * r] for r in range(w)), 1)
    send = torch.zeros(width, dtype=torch.float32, device=dev)
    send[:e1 - e0] = dP_seg[:e1 - e0]
    send = _comm(send)
    bufs = [torch.empty_like(send) for _ in range(w)] if rank == dst else None
    dist.gather(send, bufs, dst=dst)
    if rank != dst:
        return None
    P = np.zeros(int(nnz), np.float32)
    for r in range(w):
        P[b[2 * r]:b[2 * r + 1]] = bufs[r][:b[2 * r + 1] - b[2 * r]].cpu().numpy()
    return P
