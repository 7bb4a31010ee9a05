"""GPU: the rocSPARSE SDDMM baseline (include/bsmr_rocsparse.h) computes the same P as the oracle
and the engine, so bench.py's vendor_baseline compares like with like (reference counterpart:
include/cuSparseSDDMM.cuh:27-145)."""
import numpy as np
import pytest

import oracle_lib as O
from bsmr import F32, Plan, make_data, synth
from bsmr.vendor import RocsparseSddmm
from gpu_util import run_sddmm, torch_cuda

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("K", [32, 128])
def test_rocsparse_matches_oracle_and_engine(K):
    torch = torch_cuda()
    M, N, rp, ci = synth.random_rows(700, 3000, 40, seed=11, zipf=1.05, empty_frac=0.05)
    nnz = len(ci)
    A = make_data(M * K)
    B = make_data(N * K)
    c = O.CSR.from_arrays(M, N, rp, ci)
    ref = O.sddmm_cpu(c, K, A, B)
    d_rp = torch.from_numpy(rp.astype(np.int32)).cuda()
    d_ci = torch.from_numpy(ci.astype(np.int32)).cuda()
    dA = torch.from_numpy(A).cuda()
    dB = torch.from_numpy(B).cuda()
    # rocsparse_sddmm reads C even with beta = 0 (0 * NaN = NaN): P must hold finite values, as
    # the reference's P does (S's values, cuSparseSDDMM.cuh:98-101)
    dP = torch.zeros((nnz,), dtype=torch.float32, device="cuda")
    rs = RocsparseSddmm(M, N, K, nnz, d_rp.data_ptr(), d_ci.data_ptr(), dtype=F32,
                        stream=torch.cuda.current_stream().cuda_stream)
    rs(dA.data_ptr(), dB.data_ptr(), dP.data_ptr())
    torch.cuda.synchronize()
    P_vendor = dP.cpu().numpy()
    assert O.check_data(ref, P_vendor) == 0
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=288 * 1024 ** 3)
    P_engine = run_sddmm(plan, A, B, K, nnz)
    assert O.check_data(P_vendor, P_engine) == 0
