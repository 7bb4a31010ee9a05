"""Multi-GPU plumbing for row-panel sharded runs: one process per GPU over
torch.distributed (backend "nccl" = RCCL over xGMI on MI355X; "gloo" for CPU tests).

The SDDMM data path has no collective: every rank computes the outputs of its own row panels.
The only exchanges are setup (B broadcast once from rank 0) and reporting (the slowest rank's
time, per-rank counts).
"""
import os

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


def broadcast_(tensor, src=0):
    """In-place broadcast (B is generated on rank 0 and sent once, outside the timed region)."""
    import torch.distributed as dist

    dist.broadcast(tensor, src=src)
    return tensor


def max_over_ranks(value, device):
    """Max of a float over ranks (whole-job time = slowest rank)."""
    import torch
    import torch.distributed as dist

    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value, device):
    import torch
    import torch.distributed as dist

    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def panel_range(cuts, rank):
    """Row panels [p0, p1) of `rank` from the cost-model cut points (bsmr.shard_cuts)."""
    cuts = np.asarray(cuts)
    return int(cuts[rank]), int(cuts[rank + 1])
