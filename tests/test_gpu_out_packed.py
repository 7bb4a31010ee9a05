"""Packed output on the row-block launch (bsmr_tuning.out_packed): unstaged layouts
of plans with nnz <= 2^22 carry each entry's CSR position in the low 22 bits of its metadata word,
so an entry costs one 4-byte metadata load instead of two. The values must be the host SDDMM's
and bit-identical to the unpacked layout's (same arithmetic, only the store address source
changes), for the whole plan and for row-panel ranges."""
import numpy as np
import pytest

import oracle_lib as O
from bsmr import Plan, make_data, synth, tuning_from_env
from gpu_util import half_values, run_sddmm

pytestmark = pytest.mark.gpu


def _case(name):
    if name == "nips_like":
        return synth.nips_like()
    if name == "zipf":
        return synth.random_rows(900, 4000, 60, seed=21, zipf=1.1, empty_frac=0.05)
    return synth.SUITESPARSE_REBUILDS[name]()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name,K,dtype", [("nips_like", 128, 0), ("nips_like", 64, 0),
                                          ("Trefethen_20000", 64, 0), ("mycielskian14", 256, 0),
                                          ("zipf", 128, 2), ("zipf", 256, 1), ("zipf", 32, 0)])
def test_packed_output_matches_unpacked(name, K, dtype):
    M, N, rp, ci = _case(name)
    A, B = make_data(M * K), make_data(N * K)
    out = {}
    for packed in ("1", "0"):
        plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, layout="rowblock",
                    tuning=tuning_from_env({"BSMR_OUT_PACKED": packed, "BSMR_OUT_STAGED": "0"}))
        out[packed] = run_sddmm(plan, A, B, K, len(ci), dtype=dtype)
        # the plan's row-panel ranges (the shard launches) write every entry once as well
        shards = [plan.shard(K, r, 3) for r in range(3)]
        out[packed + "s"] = run_sddmm(plan, A, B, K, len(ci), panels=shards, dtype=dtype)
    Ar, Br = (A, B) if dtype == 0 else (half_values(A, dtype), half_values(B, dtype))
    ref = O.sddmm_cpu(O.CSR.from_arrays(M, N, rp, ci), K, Ar, Br)
    for k in ("1", "1s"):
        assert np.isfinite(out[k]).all()
        assert O.check_data(ref, out[k]) == 0
    assert np.array_equal(out["1"].view(np.uint32), out["0"].view(np.uint32))
    assert np.array_equal(out["1s"].view(np.uint32), out["0s"].view(np.uint32))
