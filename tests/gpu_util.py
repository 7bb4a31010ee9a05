"""Helpers for the GPU tests: device buffers through torch (plumbing only), oracle comparisons."""
import numpy as np

import oracle_lib as O


def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU test needs a HIP device"
    return torch


def run_sddmm(plan, A, B, K, nnz, panels=None, dtype=0):
    """P (fp32, NaN where not written) of the whole plan or of the given panel ranges; dtype 1/2
    rounds A and B to fp16/bf16 on the device (compare against the oracle on half_values())."""
    torch = torch_cuda()
    tdt = {0: torch.float32, 1: torch.float16, 2: torch.bfloat16}[dtype]
    dA = torch.from_numpy(np.ascontiguousarray(A, np.float32)).cuda().to(tdt)
    dB = torch.from_numpy(np.ascontiguousarray(B, np.float32)).cuda().to(tdt)
    dP = torch.full((max(nnz, 1),), float("nan"), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    if panels is None:
        plan.sddmm(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), stream=s, dtype=dtype)
    else:
        for p0, p1 in panels:
            plan.sddmm_panels(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), p0, p1, stream=s,
                              dtype=dtype)
    torch.cuda.synchronize()
    return dP.cpu().numpy()[:nnz]


def oracle_plan(M, N, rowptr, colidx, alpha, delta, free_mem):
    c = O.CSR.from_arrays(M, N, rowptr, colidx)
    bs = O.block_size(M, N, free_mem)
    rows, ncl, _ = O.row_reorder(c, np.float32(alpha), bs)
    return c, O.Plan(c, rows, ncl, np.float32(delta)), ncl


PLAN_ARRAYS = ["reorderedRows", "denseCols", "denseColOffsets", "sparseCols", "sparseColOffsets",
               "sparseValueOffsets", "blockOffsets", "blockValues", "sparseValues",
               "sparseRelativeRows", "sparseColIndices"]


def assert_plans_equal(gpu_plan, orc_plan):
    for name in PLAN_ARRAYS:
        g = gpu_plan.array(name)
        o = orc_plan.array(name)
        assert g.shape == o.shape, (name, g.shape, o.shape)
        if not np.array_equal(g, o):
            bad = np.nonzero(g != o)[0]
            raise AssertionError(f"{name}: {len(bad)} mismatches, first at {bad[:5]}: "
                                 f"gpu {g[bad[:5]]} oracle {o[bad[:5]]}")


def half_values(X, dtype):
    """X rounded (RNE) to fp16 (dtype 1) or bf16 (2), back in fp32: the values the kernel sees."""
    torch = torch_cuda()
    tdt = {1: torch.float16, 2: torch.bfloat16}[dtype]
    return torch.from_numpy(np.ascontiguousarray(X, np.float32)).to(tdt).float().numpy()
