#!/usr/bin/env python3
"""The reference's hybrid ablation on MI355X: BSMR (best alpha, delta) against "only tensor core"
(delta = 0: every tile of density > 0 on the matrix cores) and "only CUDA core" (delta = 1.1: no
tile, every entry residual) at the best alpha, per matrix and K, next to the published RTX 4090
rows of scripts/results_suiteSparse_dataset/k<K>/results_hybrid_<K>.csv.

Two steps:
  --run  (GPU box)   write the five rebuilt SuiteSparse matrices (bsmr/synth.py) as .mtx and run
                     the drop-in binary in test mode (`BSMR-sddmm -f m.mtx -t 1 -l dir/`, the
                     reference's sddmm.cu:62-118 sweep); the 140 log files per matrix go to
                     <out>/logs_<matrix>/
  --report (here)    compile the reference's own scripts/analyze_results.cpp (standalone C++)
                     from /root/reference, run it per K over each matrix's logs as
                     scripts/plot_fig_5.sh does, read its results_hybrid_<K>.csv (the table of
                     analyze_results.cpp:1122-1192) and join it with the published rows;
                     writes <out>/hybrid_table.json and prints a markdown table.

    python3 tools/hybrid_table.py --run --out gpurun_out/r04h/hybrid
    python3 tools/hybrid_table.py --report --logs tests/golden --out profiles/r04/hybrid
"""
import argparse
import csv
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sddmm-gpu_amd"))
BIN = os.path.join(ROOT, "sddmm-gpu_amd", "bin", "BSMR-sddmm")
MATRICES = ["Trefethen_20000", "Trefethen_20000b", "mycielskian14", "mycielskian15",
            "mycielskian16"]
KS = (32, 64, 128, 256)
REF = "/root/reference"
ANALYZER_SRC = os.path.join(REF, "scripts", "analyze_results.cpp")


def run(out, names):
    from bsmr import synth

    os.makedirs(out, exist_ok=True)
    for name in names:
        M, N, rp, ci = synth.SUITESPARSE_REBUILDS[name]()
        path = os.path.join(out, f"{name}.mtx")
        synth.write_mtx(path, M, N, rp, ci)
        logdir = os.path.join(out, f"logs_{name}") + "/"
        os.makedirs(logdir, exist_ok=True)
        t0 = time.time()
        r = subprocess.run([BIN, "-f", path, "-t", "1", "-l", logdir], capture_output=True,
                           text=True, timeout=900)
        os.remove(path)
        if r.returncode != 0:
            raise SystemExit(f"{name}: BSMR-sddmm failed: {r.stderr[-2000:]}")
        print(json.dumps({"matrix": name, "test_mode_s": round(time.time() - t0, 1),
                          "logs": len(os.listdir(logdir))}), flush=True)


def build_analyzer(workdir):
    exe = os.path.join(workdir, "analyze_results")
    subprocess.run(["g++", "-O1", "-o", exe, ANALYZER_SRC], check=True, capture_output=True,
                   timeout=300)
    return exe


def analyzer_hybrid(exe, logdir, K, workdir):
    """Run the reference analyzer over one matrix's K logs; its results_hybrid_<K>.csv rows."""
    d = tempfile.mkdtemp(dir=workdir)
    files = []
    for fn in sorted(os.listdir(logdir)):
        if fn.startswith(f"BSMR_k_{K}_a_"):
            shutil.copy(os.path.join(logdir, fn), os.path.join(d, fn))
            files.append(os.path.join(d, fn))
    r = subprocess.run([exe] + files, capture_output=True, text=True, timeout=120, cwd=d)
    if r.returncode != 0:
        raise RuntimeError(f"analyzer failed on {logdir} K={K}: {r.stderr[-500:]}")
    return list(csv.DictReader(open(os.path.join(d, f"results_hybrid_{K}.csv"))))


def published_rows(name, K):
    """(line number, row) of the matrix in the reference's published results_hybrid_<K>.csv."""
    path = os.path.join(REF, "scripts", "results_suiteSparse_dataset", f"k{K}",
                        f"results_hybrid_{K}.csv")
    with open(path) as f:
        lines = f.read().splitlines()
    hdr = lines[0].split(",")
    for i, line in enumerate(lines[1:], start=2):
        v = line.split(",")
        if v[0].endswith(f"/{name}.mtx"):
            return i, dict(zip(hdr, v)), os.path.relpath(path, REF)
    return None, None, os.path.relpath(path, REF)


def report(logs_root, out, prefix):
    os.makedirs(out, exist_ok=True)
    work = tempfile.mkdtemp(prefix="hybrid_")
    exe = build_analyzer(work)
    rows = []
    for name in MATRICES:
        logdir = os.path.join(logs_root, f"{prefix}{name}")
        for K in KS:
            hyb = analyzer_hybrid(exe, logdir, K, work)
            assert len(hyb) == 1, (name, K, hyb)
            h = hyb[0]
            line, pub, src = published_rows(name, K)
            b, tc, cc = float(h["BSMR"]), float(h["BSMR_Only_Tensor_core"]), float(h["BSMR_Only_CUDA_Core"])
            row = {"matrix": name, "K": K, "alpha": float(h["alpha"]),
                   "mi355x_bsmr": b, "mi355x_only_tensor_core": tc, "mi355x_only_cuda_core": cc,
                   "mi355x_hybrid_over_tc": round(b / tc, 3) if tc else None,
                   "mi355x_hybrid_over_cc": round(b / cc, 3) if cc else None}
            if pub:
                pb, ptc, pcc = (float(pub["BSMR"]), float(pub["BSMR_Only_Tensor_core"]),
                                float(pub["BSMR_Only_CUDA_Core"]))
                row.update({"rtx4090_alpha": float(pub["alpha"]), "rtx4090_bsmr": pb,
                            "rtx4090_only_tensor_core": ptc, "rtx4090_only_cuda_core": pcc,
                            "rtx4090_hybrid_over_tc": round(pb / ptc, 3) if ptc else None,
                            "rtx4090_hybrid_over_cc": round(pb / pcc, 3) if pcc else None,
                            "published": f"{src}:{line}"})
            rows.append(row)
    shutil.rmtree(work, ignore_errors=True)
    res = {"source": "reference scripts/analyze_results.cpp (compiled from source) over the "
                     "MI355X test-mode logs of each matrix; published rows from "
                     "scripts/results_suiteSparse_dataset/k<K>/results_hybrid_<K>.csv",
           "columns": "BSMR = best bsmr_gflops over alpha x delta; only tensor core = delta 0 "
                      "at that alpha; only CUDA core = delta 1.1 at that alpha "
                      "(analyze_results.cpp:1143-1158)",
           "rows": rows}
    with open(os.path.join(out, "hybrid_table.json"), "w") as f:
        json.dump(res, f, indent=1)
    print("| matrix | K | MI355X BSMR | δ=0 (MFMA tiles) | δ=1.1 (residual only) | hybrid/δ0 | "
          "hybrid/δ1.1 | RTX 4090 BSMR | δ=0 | δ=1.1 | hybrid/δ0 | hybrid/δ1.1 | published row |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|---|")
    for r in rows:
        print(f"| {r['matrix']} | {r['K']} | {r['mi355x_bsmr']:.0f} | {r['mi355x_only_tensor_core']:.0f} "
              f"| {r['mi355x_only_cuda_core']:.0f} | {r['mi355x_hybrid_over_tc']} | "
              f"{r['mi355x_hybrid_over_cc']} | {r.get('rtx4090_bsmr', '')} | "
              f"{r.get('rtx4090_only_tensor_core', '')} | {r.get('rtx4090_only_cuda_core', '')} | "
              f"{r.get('rtx4090_hybrid_over_tc', '')} | {r.get('rtx4090_hybrid_over_cc', '')} | "
              f"`{r.get('published', '')}` |")
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--run", action="store_true")
    ap.add_argument("--report", action="store_true")
    ap.add_argument("--out", default="gpurun_out/hybrid")
    ap.add_argument("--logs", default=None, help="--report: directory holding the log dirs")
    ap.add_argument("--prefix", default="mi355x_testmode_",
                    help="--report: log directory name prefix (logs_ for a --run output)")
    ap.add_argument("--matrices", default=",".join(MATRICES))
    args = ap.parse_args()
    if args.run:
        run(args.out, args.matrices.split(","))
    if args.report:
        report(args.logs or args.out, args.out, args.prefix)


if __name__ == "__main__":
    main()
