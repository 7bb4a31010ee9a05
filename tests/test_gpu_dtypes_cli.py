"""GPU: fp16/bf16 inputs (configs C3/C5) and the BSMR-sddmm drop-in binary."""
import os
import re
import subprocess

import numpy as np
import pytest

import oracle_lib as O
from bsmr import BF16, F16, Plan, make_data, synth, tuning_from_env
from gpu_util import torch_cuda

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "sddmm-gpu_amd", "bin", "BSMR-sddmm")
# the same CLI built with -DBSMR_FAULT_INJECT (honours BSMR_VALIDATE_CORRUPT); test use only
BIN_FI = os.path.join(ROOT, "sddmm-gpu_amd", "bin", "BSMR-sddmm-faultinject")
FREE = 288 * 1024 ** 3


def to_bf16_bits(x):
    b = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.uint64)
    r = ((b + 0x7FFF + ((b >> 16) & 1)) >> 16).astype(np.uint16)
    return r, (r.astype(np.uint32) << 16).view(np.float32)


def to_f16_bits(x):
    h = np.ascontiguousarray(x, np.float32).astype(np.float16)
    return h.view(np.uint16), h.astype(np.float32)


def run_half(plan, Ab, Bb, K, nnz, dtype):
    torch = torch_cuda()
    dA = torch.from_numpy(Ab.view(np.int16)).cuda()
    dB = torch.from_numpy(Bb.view(np.int16)).cuda()
    dP = torch.full((nnz,), float("nan"), dtype=torch.float32, device="cuda")
    plan.sddmm(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(),
               stream=torch.cuda.current_stream().cuda_stream, dtype=dtype)
    torch.cuda.synchronize()
    return dP.cpu().numpy()


@pytest.mark.parametrize("dtype", [F16, BF16])
@pytest.mark.parametrize("K", [32, 96, 128, 256, 512])
@pytest.mark.parametrize("case", ["blocky", "zipf", "banded"])
@pytest.mark.parametrize("layout", ["rowblock", "colmajor"])
def test_half_inputs_checkdata(dtype, K, case, layout):
    """fp16/bf16 A/B: row-block kernel for K = 128/256 (rows of 256/512 bytes), column-major
    otherwise or when forced."""
    if case == "blocky":
        M, N, rp, ci = synth.block_mask(512, 16, 0.1, seed=7)
    elif case == "zipf":
        M, N, rp, ci = synth.random_rows(400, 3000, 50, seed=8, zipf=1.1)
    else:  # cop20k-like banded FEM: many small row blocks, several piece phases per item
        M, N, rp, ci = synth.banded_fem_like(6000, 22, seed=3, band=48)
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE, layout=layout)
    A = make_data(M * K)
    B = make_data(N * K)
    conv = to_bf16_bits if dtype == BF16 else to_f16_bits
    Ab, Ar = conv(A)
    Bb, Br = conv(B)
    P = run_half(plan, Ab, Bb, K, len(ci), dtype)
    assert np.isfinite(P).all()
    # oracle in fp32 on the same rounded values: half x half products are exact in fp32
    ref = O.sddmm_cpu(O.CSR.from_arrays(M, N, rp, ci), K, Ar, Br)
    assert O.check_data(ref, P) == 0


@pytest.mark.parametrize("case,K,dtype,force", [
    ("uniform300", 256, F16, False),    # 20 % dense, ragged tiles (300 = 2 x 128 + 44)
    ("uniform300", 128, BF16, False),
    ("uniform300", 512, F16, False),
    ("uniform300", 64, F16, False),     # one k-chunk: every prefetch re-reads it
    ("uniform300", 320, BF16, False),   # 5 chunks: the 4-stage loop leaves mid-way
    ("zipf", 128, BF16, True),          # sparse pattern forced dense: empty tiles skipped
    ("zipf", 256, F16, True),
])
def test_dense_sampled_half(case, K, dtype, force):
    """The dense-sampled MFMA launch (whole 128 x 128 tiles of A B^T, sampled) for fp16/bf16
    patterns above the density threshold (layout auto), against the oracle on the rounded
    values."""
    tun = tuning_from_env({"BSMR_DENSE_MIN": "0"} if force else {})
    if case == "uniform300":
        M, N, rp, ci = synth.uniform_mask(300, 0.2, seed=5)
    elif case == "zipf":
        M, N, rp, ci = synth.random_rows(400, 3000, 50, seed=8, zipf=1.1)
    else:
        M, N, rp, ci = synth.block_mask(512, 16, 0.1, seed=7)
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE, tuning=tun)
    conv = to_bf16_bits if dtype == BF16 else to_f16_bits
    Ab, Ar = conv(make_data(M * K))
    Bb, Br = conv(make_data(N * K)[::-1].copy())
    P = run_half(plan, Ab, Bb, K, len(ci), dtype)
    assert np.isfinite(P).all()
    ref = O.sddmm_cpu(O.CSR.from_arrays(M, N, rp, ci), K, Ar, Br)
    assert O.check_data(ref, P) == 0


@pytest.mark.parametrize("env,K,dtype", [
    ({"BSMR_DENSE_KS": "1"}, 256, F16),    # four waves, 64 x 64 quadrants (>= 512 tiles by default)
    ({"BSMR_DENSE_KS": "1"}, 320, BF16),
    ({"BSMR_DENSE_NS": "3"}, 320, BF16),   # eight waves, 3-5 LDS stages (BSMR_DENSE_NS)
    ({"BSMR_DENSE_NS": "4"}, 256, F16),
    ({"BSMR_DENSE_NS": "5"}, 128, BF16),   # fewer chunks than stages
    ({"BSMR_DENSE_NS": "5"}, 512, F16),
])
def test_dense_sampled_variants(env, K, dtype):
    """Every wave/stage form of the dense-sampled launch (sddmm_dense.hip launch_dense) gives the
    oracle's values on a ragged 300 x 300 pattern (edge tiles read clamped rows)."""
    M, N, rp, ci = synth.uniform_mask(300, 0.2, seed=11)
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE,
                tuning=tuning_from_env(env))
    conv = to_bf16_bits if dtype == BF16 else to_f16_bits
    Ab, Ar = conv(make_data(M * K))
    Bb, Br = conv(make_data(N * K)[::-1].copy())
    P = run_half(plan, Ab, Bb, K, len(ci), dtype)
    assert np.isfinite(P).all()
    ref = O.sddmm_cpu(O.CSR.from_arrays(M, N, rp, ci), K, Ar, Br)
    assert O.check_data(ref, P) == 0


def test_dlmc_like_bf16_k512():
    M, N, rp, ci = synth.uniform_mask(2048, 0.1, seed=7)
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE)
    K = 512
    Ab, Ar = to_bf16_bits(make_data(M * K))
    Bb, Br = to_bf16_bits(make_data(N * K))
    P = run_half(plan, Ab, Bb, K, len(ci), BF16)
    ref = O.sddmm_cpu(O.CSR.from_arrays(M, N, rp, ci), K, Ar, Br)
    assert O.check_data(ref, P) == 0


def _log_fields(text):
    return dict(re.findall(r"\[([A-Za-z_][A-Za-z_ ]*?)\s*: ([^\]]*)\]", text))


def test_cli_default_run_log(tmp_path):
    M, N, rp, ci = synth.random_rows(600, 2000, 40, seed=9, zipf=1.05)
    path = str(tmp_path / "s.mtx")
    synth.write_mtx(path, M, N, rp, ci)
    r = subprocess.run([BIN, "-f", path, "-k", "64", "-a", "0.3", "-d", "0.3"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert f"sparseMatrix::CSR initialize from file : {path}" in r.stdout
    f = _log_fields(r.stdout)
    assert f["K"] == "64" and f["M"] == str(M) and f["NNZ"] == str(len(ci))
    assert f["matrixA storageOrder"] == "row_major" and f["matrixB storageOrder"] == "col_major"
    assert f["bsmr_alpha"] == "0.30" and f["bsmr_delta"] == "0.30"
    # reorder statistics equal the oracle's
    c = O.CSR.from_arrays(M, N, rp, ci)
    rows, ncl, _ = O.row_reorder(c, np.float32(0.3), O.block_size(M, N, FREE))
    s = O.Plan(c, rows, ncl, np.float32(0.3)).stats()
    assert int(f["bsmr_numClusters"]) == ncl
    assert int(f["NumRowPanel"]) == s["numRowPanels"]
    assert int(f["bsmr_numDenseBlock"]) == s["numDenseBlock"]
    assert int(f["bsmr_numSparseData"]) == s["numSparseData"]
    assert float(f["bsmr_gflops"]) > 0
    # the reference analysis script's parser (analyze_results.cpp getValue) finds the key
    assert re.search(r"\[bsmr_gflops : [0-9.]+\]", r.stdout)


@pytest.mark.parametrize("fmt", ["smtx", "snap"])
def test_cli_other_formats(tmp_path, fmt):
    """.smtx (DLMC) and SNAP .txt inputs through the CLI's suffix dispatch: checkData passes."""
    M, N, rp, ci = synth.random_rows(400, 400, 30, seed=12, zipf=1.05)
    if fmt == "smtx":
        path = str(tmp_path / "s.smtx")
        synth.write_smtx(path, M, N, rp, ci)
    else:
        path = str(tmp_path / "s.txt")
        synth.write_snap(path, M, rp, ci)
    r = subprocess.run([BIN, "-f", path, "-k", "128"], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, BSMR_VALIDATE="1"))
    assert r.returncode == 0, r.stderr
    assert f"sparseMatrix::CSR initialize From file : {path}" in r.stdout
    f = _log_fields(r.stdout)
    assert f["NNZ"] == str(len(ci)) and f["K"] == "128"
    # the validate path ran (host SDDMM + checkData of the loaded matrix) and passed
    assert "| Pass! Result validates successfully." in r.stdout
    assert "NO PASS" not in r.stdout


def test_cli_positional_and_failure(tmp_path):
    M, N, rp, ci = synth.random_rows(100, 300, 10, seed=10)
    path = str(tmp_path / "p.mtx")
    synth.write_mtx(path, M, N, rp, ci)
    r = subprocess.run([BIN, path, "32"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "[K : 32]" in r.stdout
    bad = str(tmp_path / "bad.mtx")
    open(bad, "w").write("%x\n2 2 2\n1 1 1\n1 1 1\n")
    r = subprocess.run([BIN, "-f", bad], capture_output=True, text=True, timeout=60)
    assert r.returncode == 255
    assert "Error, matrix S initialize failed." in r.stderr


def test_cli_test_mode_writes_reference_log_files(tmp_path):
    M, N, rp, ci = synth.random_rows(200, 800, 20, seed=11)
    path = str(tmp_path / "t.mtx")
    synth.write_mtx(path, M, N, rp, ci)
    logdir = str(tmp_path) + "/"
    r = subprocess.run([BIN, "-f", path, "-t", "1", "-l", logdir], capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0, r.stderr
    names = sorted(os.listdir(tmp_path))
    logs = [n for n in names if n.startswith("BSMR_k_")]
    assert len(logs) == 5 * 7 * 4
    assert "BSMR_k_128_a_0.3_d_0.3.log" in logs and "BSMR_k_32_a_0.1_d_0.log" in logs
    assert "BSMR_k_256_a_0.9_d_1.1.log" in logs
    text = open(os.path.join(tmp_path, "BSMR_k_128_a_0.3_d_0.3.log")).read()
    assert text.startswith("\n---New data---\n")
    assert _log_fields(text)["bsmr_delta"] == "0.30"


@pytest.mark.parametrize("dtype", [F16, BF16])
def test_half_k1024_rowblock(dtype):
    """2 KiB rows (K = 1024 half): the 16-lanes-per-entry row-block kernel."""
    M, N, rp, ci = synth.random_rows(700, 2500, 60, seed=21, zipf=1.1)
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE)
    K = 1024
    conv = to_bf16_bits if dtype == BF16 else to_f16_bits
    Ab, Ar = conv(make_data(M * K))
    Bb, Br = conv(make_data(N * K))
    P = run_half(plan, Ab, Bb, K, len(ci), dtype)
    assert plan.stats()["rb_items"][4] > 0
    ref = O.sddmm_cpu(O.CSR.from_arrays(M, N, rp, ci), K, Ar, Br)
    assert O.check_data(ref, P) == 0


def _oracle_report(n, n_err_vals=None):
    """checkData's framed text for n values as the oracle prints it (child process: stdout)."""
    import sys
    import textwrap
    code = textwrap.dedent(f"""
        import sys, numpy as np
        sys.path[:0] = {sys.path!r}
        import oracle_lib as O
        a = np.zeros({n}, np.float32)
        O.check_data(a, a, verbose=True)
    """)
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                          check=True, timeout=120).stdout


@pytest.mark.parametrize("corrupt", [0, 7])
def test_cli_validate_checkdata_surface(tmp_path, corrupt):
    """BSMR_VALIDATE=1 (the reference's VALIDATE build, sddmm.cu:34-59): the host SDDMM of the same
    operands, checkData's framed block before the log, and on a deliberately corrupted P
    (BSMR_VALIDATE_CORRUPT=n adds 1 to the first n GPU values; only the test build BIN_FI has that
    hook, the release binary ignores the variable) the errors and the NO PASS line."""
    M, N, rp, ci = synth.random_rows(500, 1500, 30, seed=13, zipf=1.05)
    path = str(tmp_path / "v.mtx")
    synth.write_mtx(path, M, N, rp, ci)
    env = dict(os.environ, BSMR_VALIDATE="1")
    if corrupt:
        env["BSMR_VALIDATE_CORRUPT"] = str(corrupt)
        # the release binary has no fault-injection hook: the variable changes nothing
        r = subprocess.run([BIN, "-f", path, "-k", "64"], capture_output=True, text=True,
                           timeout=300, env=env)
        assert r.returncode == 0 and "NO PASS" not in r.stdout, r.stderr
    r = subprocess.run([BIN_FI if corrupt else BIN, "-f", path, "-k", "64"], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    out = r.stdout
    head = "check cpu sddmm and BSMR sddmm: \n"
    assert head in out
    block = out[out.index(head) + len(head):]
    block = block[:block.index("|----------------------------------------------------------------|\n") + 67]
    # the block precedes the log (sddmm() validates before main prints the log)
    assert out.index(head) < out.index("[bsmr_gflops : ")
    nnz = len(ci)
    if not corrupt:
        assert block == _oracle_report(nnz)
        assert "NO PASS" not in out
        return
    lines = block.splitlines()
    assert lines[:4] == _oracle_report(nnz).splitlines()[:4]
    A = make_data(M * 64)
    B = make_data(N * 64)
    ref = O.sddmm_cpu(O.CSR.from_arrays(M, N, rp, ci), 64, A, B)
    errs = [x for x in lines if x.startswith("| Error : idx = ")]
    assert len(errs) == corrupt
    for i, x in enumerate(errs):
        m = re.match(r"\| Error : idx = (\d+), data1 = ([-0-9.]+), data2 = ([-0-9.]+), "
                     r"difference = ([-0-9.]+)$", x)
        assert m and int(m.group(1)) == i
        assert m.group(2) == f"{ref[i]:f}"
        assert abs(float(m.group(3)) - (ref[i] + 1.0)) < 1e-3
    rate = np.float32(corrupt) / np.float32(nnz) * np.float32(100)
    assert f"| No Pass! Inconsistent data! {corrupt} errors! Error rate : {rate:2.2f}%" in lines
    assert f"[checkData : NO PASS Error rate : {rate:2.2f}%]" in out
