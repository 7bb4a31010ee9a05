"""f1: the reference's own log consumer reads MI355X test-mode logs unchanged,
and its hybrid ablation table (BSMR / delta 0 "only tensor core" / delta 1.1 "only CUDA core",
analyze_results.cpp:1122-1192) is the one DESIGN.md §8.1 reports.

The fixtures are the 140 log files per matrix that the drop-in binary wrote in test mode on
MI355X (`BSMR-sddmm -f <matrix>.mtx -t 1 -l dir/`, sddmm.cu:62-118: 5 alpha x 7 delta x
K in {32, 64, 128, 256}; tools/hybrid_table.py --run) for the five SuiteSparse matrices the
engine rebuilds exactly (bsmr/synth.py). The reference's scripts/analyze_results.cpp is compiled
here from its own source with g++ (it is standalone C++, analyze_results.cpp:1-14) and run per K
as scripts/plot_fig_5.sh does; it must accept the log set (SettingInformation::initInformation,
analyze_results.cpp:122-160, rejects logs whose settings differ), its results_<K>.csv must carry
the best bsmr_gflops of the sweep in the BSMR column (analyze_results.cpp:283-345, 785-830), and
its results_hybrid_<K>.csv must equal the MI355X columns of tests/golden/mi355x_hybrid_table.json
(written by tools/hybrid_table.py --report from the same logs). Skipped when /root/reference is
absent (the GPU box)."""
import csv
import json
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = "/root/reference/scripts/analyze_results.cpp"
GOLDEN = os.path.join(ROOT, "tests", "golden")
TABLE = os.path.join(GOLDEN, "mi355x_hybrid_table.json")
SIZES = {"Trefethen_20000": ("20000", "20000", "287233"),
         "Trefethen_20000b": ("19999", "19999", "287217"),
         "mycielskian14": ("12287", "12287", "1847756"),
         "mycielskian15": ("24575", "24575", "5555555"),
         "mycielskian16": ("49151", "49151", "16691240")}
MATRICES = [m for m in SIZES if os.path.isdir(os.path.join(GOLDEN, f"mi355x_testmode_{m}"))]


def logs(name):
    return os.path.join(GOLDEN, f"mi355x_testmode_{name}")


@pytest.fixture(scope="module")
def analyzer(tmp_path_factory):
    if not os.path.exists(SRC) or shutil.which("g++") is None:
        pytest.skip("reference analyze_results.cpp (or g++) not available")
    exe = str(tmp_path_factory.mktemp("ar") / "analyze_results")
    subprocess.run(["g++", "-O1", "-o", exe, SRC], check=True, capture_output=True, timeout=300)
    return exe


def _best(name, K):
    best = 0.0
    for fn in os.listdir(logs(name)):
        m = re.match(r"BSMR_k_(\d+)_a_([\d.]+)_d_([\d.]+)\.log$", fn)
        if m and int(m.group(1)) == K:
            text = open(os.path.join(logs(name), fn)).read()
            best = max(best, max(float(v) for v in re.findall(r"\[bsmr_gflops : ([0-9.]+)\]", text)))
    return best


def test_all_five_matrices_have_fixtures():
    assert MATRICES == list(SIZES)


@pytest.mark.parametrize("name", MATRICES)
def test_fixture_set_complete(name):
    names = [n for n in os.listdir(logs(name)) if n.startswith("BSMR_k_")]
    assert len(names) == 5 * 7 * 4
    for n in names:
        text = open(os.path.join(logs(name), n)).read()
        assert text.startswith("\n---New data---\n") and "[bsmr_gflops : " in text


@pytest.mark.parametrize("K", [32, 64, 128, 256])
@pytest.mark.parametrize("name", MATRICES)
def test_reference_analyzer_consumes_logs(analyzer, tmp_path, name, K):
    files = []
    for fn in sorted(os.listdir(logs(name))):
        if fn.startswith(f"BSMR_k_{K}_a_"):
            shutil.copy(os.path.join(logs(name), fn), tmp_path / fn)
            files.append(str(tmp_path / fn))
    assert len(files) == 35
    r = subprocess.run([analyzer] + files, capture_output=True, text=True, timeout=120,
                       cwd=tmp_path)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    rows = list(csv.DictReader(open(tmp_path / f"results_{K}.csv")))
    assert len(rows) == 1  # one matrix
    row = rows[0]
    assert row["file"].endswith(f"{name}.mtx")
    assert (row["M"], row["N"], row["NNZ"], row["K"]) == SIZES[name] + (str(K),)
    assert abs(float(row["BSMR"]) - _best(name, K)) <= 1e-3 * _best(name, K)
    # the hybrid table (delta = 0 "only tensor core" / delta > 1 "only CUDA core") is written
    # too, and is the table DESIGN.md §8.1 reports
    hyb = list(csv.DictReader(open(tmp_path / f"results_hybrid_{K}.csv")))
    assert len(hyb) == 1 and float(hyb[0]["BSMR"]) == float(row["BSMR"])
    table = {(t["matrix"], t["K"]): t for t in json.load(open(TABLE))["rows"]}
    t = table[(name, K)]
    assert float(hyb[0]["alpha"]) == pytest.approx(t["alpha"])
    assert float(hyb[0]["BSMR"]) == pytest.approx(t["mi355x_bsmr"], rel=1e-6)
    assert float(hyb[0]["BSMR_Only_Tensor_core"]) == pytest.approx(t["mi355x_only_tensor_core"],
                                                                    rel=1e-6)
    assert float(hyb[0]["BSMR_Only_CUDA_Core"]) == pytest.approx(t["mi355x_only_cuda_core"],
                                                                  rel=1e-6)
