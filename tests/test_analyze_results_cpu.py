"""f1: the reference's own log consumer reads MI355X test-mode logs unchanged.

The fixtures are the 140 log files the drop-in binary wrote in test mode on MI355X
(`BSMR-sddmm -f Trefethen_20000.mtx -t 1 -l dir/`, sddmm.cu:62-118: 5 alpha x 7 delta x
K in {32, 64, 128, 256}; tools/hybrid_table.py --run). The reference's scripts/analyze_results.cpp is compiled
here from its own source with g++ (it is standalone C++, analyze_results.cpp:1-14) and run per K as
scripts/plot_fig_5.sh does; it must accept the log set (SettingInformation::initInformation,
analyze_results.cpp:122-160, rejects logs whose settings differ) and its results_<K>.csv must carry
the best bsmr_gflops of the sweep in the BSMR column (analyze_results.cpp:283-345, 785-830).
Skipped when /root/reference is absent (the GPU box)."""
import csv
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = "/root/reference/scripts/analyze_results.cpp"
LOGS = os.path.join(ROOT, "tests", "golden", "mi355x_testmode_Trefethen_20000")


@pytest.fixture(scope="module")
def analyzer(tmp_path_factory):
    if not os.path.exists(SRC) or shutil.which("g++") is None:
        pytest.skip("reference analyze_results.cpp (or g++) not available")
    exe = str(tmp_path_factory.mktemp("ar") / "analyze_results")
    subprocess.run(["g++", "-O1", "-o", exe, SRC], check=True, capture_output=True, timeout=300)
    return exe


def _best(K):
    best = 0.0
    for fn in os.listdir(LOGS):
        m = re.match(r"BSMR_k_(\d+)_a_([\d.]+)_d_([\d.]+)\.log$", fn)
        if m and int(m.group(1)) == K:
            text = open(os.path.join(LOGS, fn)).read()
            best = max(best, max(float(v) for v in re.findall(r"\[bsmr_gflops : ([0-9.]+)\]", text)))
    return best


def test_fixture_set_complete():
    names = [n for n in os.listdir(LOGS) if n.startswith("BSMR_k_")]
    assert len(names) == 5 * 7 * 4
    for n in names:
        text = open(os.path.join(LOGS, n)).read()
        assert text.startswith("\n---New data---\n") and "[bsmr_gflops : " in text


@pytest.mark.parametrize("K", [32, 64, 128, 256])
def test_reference_analyzer_consumes_logs(analyzer, tmp_path, K):
    files = []
    for fn in sorted(os.listdir(LOGS)):
        if fn.startswith(f"BSMR_k_{K}_a_"):
            shutil.copy(os.path.join(LOGS, fn), tmp_path / fn)
            files.append(str(tmp_path / fn))
    assert len(files) == 35
    r = subprocess.run([analyzer] + files, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    rows = list(csv.DictReader(open(tmp_path / f"results_{K}.csv")))
    assert len(rows) == 1  # one matrix
    row = rows[0]
    assert row["file"].endswith("Trefethen_20000.mtx")
    assert (row["M"], row["N"], row["NNZ"], row["K"]) == ("20000", "20000", "287233", str(K))
    assert abs(float(row["BSMR"]) - _best(K)) <= 1e-3 * _best(K)
    # the hybrid table (delta = 0 "only tensor core" / delta > 1 "only CUDA core") is written too
    hyb = list(csv.DictReader(open(tmp_path / f"results_hybrid_{K}.csv")))
    assert hyb and all(float(h["BSMR"]) == float(row["BSMR"]) for h in hyb)
