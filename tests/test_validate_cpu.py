"""CPU checks of the product-side validation path (csrc/host_check.cpp, no device calls):
bsmr_sddmm_cpu equals the oracle's restatement of host.cpp:45-76 bit for bit, and
bsmr_check_data prints checkData's framed report (checkData.hpp:44-79) exactly as the oracle's
restatement does, including the NO PASS branch on a corrupted P."""
import subprocess
import sys
import textwrap

import numpy as np
import pytest

import bsmr
import oracle_lib as O
from bsmr import synth


@pytest.mark.parametrize("K,threads", [(32, 1), (64, 3), (128, 0), (48, 8)])
def test_sddmm_cpu_bit_exact_vs_oracle(K, threads):
    M, N, rp, ci = synth.random_rows(500, 3000, 40, seed=31, zipf=1.1, empty_frac=0.05)
    A = bsmr.make_data(M * K)
    B = bsmr.make_data(N * K)
    P = bsmr.sddmm_cpu(M, N, rp, ci, K, A, B, threads=threads)
    ref = O.sddmm_cpu(O.CSR.from_arrays(M, N, rp, ci), K, A, B)
    assert np.array_equal(P.view(np.uint32), ref.view(np.uint32))


def test_check_one_rule():
    L = bsmr.lib()
    for a, b in [(1.0, 1.0), (1.0, 1.0009), (1.0, 1.0011), (0.0, 9e-6), (0.0, 2e-5),
                 (1e-4, 1.5e-4), (-3.0, 3.0), (1e6, 1e6 + 900.0), (1e6, 1e6 + 1100.0)]:
        assert L.bsmr_check_one(a, b) == O.lib().orc_check_one(a, b), (a, b)


def _report(mod, n_err):
    """stdout of check_data(verbose) of `mod` (bsmr or the oracle) in a child process."""
    code = textwrap.dedent(f"""
        import sys, numpy as np
        sys.path[:0] = {sys.path!r}
        import bsmr, oracle_lib as O
        a = np.linspace(-5, 5, 1000).astype(np.float32)
        b = a.copy()
        b[:{n_err}] += 1.0
        if "{mod}" == "bsmr":
            n = bsmr.check_data(a, b, verbose=True)
        else:
            n = O.check_data(a, b, verbose=True)
        print("errors", n)
    """)
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                          check=True, timeout=120).stdout


@pytest.mark.parametrize("n_err", [0, 3, 25])
def test_check_data_report_text_matches_oracle(n_err):
    mine = _report("bsmr", n_err)
    ref = _report("oracle", n_err)
    assert mine == ref
    assert mine.startswith("|---------------------------check data---------------------------|\n")
    if n_err:
        assert f"No Pass! Inconsistent data! {n_err} errors!" in mine
        assert mine.count("| Error : idx = ") == min(n_err, 9)
    else:
        assert "| Pass! Result validates successfully." in mine
