#!/usr/bin/env python3
"""MI355X vs the reference's published RTX 4090 numbers on the same matrices.

The five SuiteSparse matrices of the reference's sweep that bsmr/synth.py rebuilds exactly
(Trefethen_20000, Trefethen_20000b, mycielskian14/15/16; their reorder statistics equal the
reference logs, tests/test_oracle_golden.py) are written as .mtx files and run through the
drop-in binary in the reference's own test mode (`BSMR-sddmm -f <m>.mtx -t 1 -l <dir>/`,
sddmm.cu:62-118: 5 alpha x 7 delta x K in {32, 64, 128, 256}, 10 timed iterations each, the
reference's log files). The per-K figure is the best bsmr_gflops over the 35 (alpha, delta)
settings, the rule of the reference's analysis (analyze_results.cpp:283-345). K = 512
(north_star) is not in the test-mode sweep: it is measured through the C ABI with the same
protocol (plan per alpha, recolumn per delta, 10 back-to-back launches timed by HIP events).

Published numbers: tests/golden/reference_published_gflops.json (extracted from the reference's
results_<K>.csv by tools/extract_reference_published.py).

    python3 tools/suitesparse_compare.py --out gpurun_out/ss [--matrices a,b] [--no-k512]
"""
import argparse
import json
import os
import re
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sddmm-gpu_amd"))
BIN = os.path.join(ROOT, "sddmm-gpu_amd", "bin", "BSMR-sddmm")
ALPHAS = [0.1, 0.3, 0.5, 0.7, 0.9]
DELTAS = [0.0, 0.1, 0.3, 0.5, 0.7, 0.9, 1.1]


def parse_logs(logdir):
    """{(K, alpha, delta): (gflops, sddmm_ms)} from the test-mode log files of one matrix."""
    out = {}
    for fn in os.listdir(logdir):
        m = re.match(r"BSMR_k_(\d+)_a_([\d.]+)_d_([\d.]+)\.log$", fn)
        if not m:
            continue
        text = open(os.path.join(logdir, fn)).read()
        g = re.findall(r"\[bsmr_gflops : ([0-9.eE+-]+|inf|nan)\]", text)
        t = re.findall(r"\[bsmr_sddmm : ([0-9.eE+-]+)\]", text)
        out[(int(m.group(1)), float(m.group(2)), float(m.group(3)))] = (float(g[-1]), float(t[-1]))
    return out


def k512(name, M, N, rp, ci, iters=10):
    """Best GFLOP/s over alpha x delta at K = 512 (fp32), the test-mode protocol via the C ABI."""
    import torch

    from bsmr import Plan, make_data

    K = 512
    dA = torch.from_numpy(make_data(M * K)).cuda()
    dB = torch.from_numpy(make_data(N * K)).cuda()
    dP = torch.zeros(len(ci), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream()
    best = None
    grid = {}
    for a in ALPHAS:
        plan = Plan(M, N, rp, ci, alpha=a, delta=DELTAS[0])
        for d in DELTAS:
            plan.recolumn(d)
            plan.sddmm(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), stream=s.cuda_stream)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(iters):
                plan.sddmm(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), stream=s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / iters
            gf = 2.0 * len(ci) * K / (ms * 1e6)
            grid[f"{a}/{d}"] = round(gf, 2)
            if best is None or gf > best[0]:
                best = (gf, a, d, ms)
        del plan
    return {"gflops": round(best[0], 2), "alpha": best[1], "delta": best[2],
            "ms": round(best[3], 5), "grid": grid}


def retime_and_cpu(M, N, rp, ci, K, alpha, delta, iters=100):
    """The best setting re-timed through the C ABI (HIP events over `iters` back-to-back launches,
    the log prints bsmr_sddmm with 2 decimals only), its HBM roofline fraction (algorithmic bytes
    4K(M+N) + 8 nnz + 4(M+1), SURVEY.md §8d, against 8 TB/s) and the same-box CPU rate: the
    product's OpenMP host SDDMM (host.cpp:45-76 restated) on all host cores, median of 3 after a
    warm-up, with checkData of the GPU P against it."""
    import statistics

    import torch

    from bsmr import Plan, check_data, make_data, sddmm_cpu

    A = make_data(M * K)
    B = make_data(N * K)
    dA = torch.from_numpy(A).cuda()
    dB = torch.from_numpy(B).cuda()
    dP = torch.zeros(len(ci), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream()
    plan = Plan(M, N, rp, ci, alpha=alpha, delta=delta)
    for _ in range(3):
        plan.sddmm(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), stream=s.cuda_stream)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        plan.sddmm(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), stream=s.cuda_stream)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    nnz = len(ci)
    flops = 2.0 * nnz * K
    bytes_alg = 4.0 * K * (M + N) + 8.0 * nnz + 4.0 * (M + 1)
    # the box's CPU share: at most 16 threads (a box has exported OMP_NUM_THREADS=256, and all of
    # os.cpu_count() would oversubscribe a shared host)
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)))
    sddmm_cpu(M, N, rp, ci, K, A, B, threads=threads)
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        P = sddmm_cpu(M, N, rp, ci, K, A, B, threads=threads)
        ts.append(time.perf_counter() - t0)
    cpu_s = statistics.median(ts)
    return {"event_ms": round(ms, 5), "event_gflops": round(flops / (ms * 1e-3) / 1e9, 2),
            "roofline_frac": round(bytes_alg / (ms * 1e-3) / 8e12, 4),
            "bytes_alg": bytes_alg,
            "cpu_gflops": round(flops / cpu_s / 1e9, 2), "cpu_ms": round(cpu_s * 1e3, 3),
            "cpu_threads": threads,
            "checkData_errors_gpu_vs_cpu": check_data(P, dP.cpu().numpy())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/ss")
    ap.add_argument("--matrices", default="Trefethen_20000,Trefethen_20000b,mycielskian14,"
                                          "mycielskian15,mycielskian16")
    ap.add_argument("--no-k512", action="store_true")
    ap.add_argument("--keep-mtx", action="store_true", help="keep the .mtx files (rocprof pass)")
    args = ap.parse_args()
    from bsmr import synth

    os.makedirs(args.out, exist_ok=True)
    pub = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_published_gflops.json")))
    published = {(r["matrix"], r["K"]): r for r in pub["rows"]}
    cpu = ""
    try:
        cpu = [x.split(":", 1)[1].strip() for x in open("/proc/cpuinfo")
               if x.startswith("model name")][0]
    except (OSError, IndexError):
        pass
    result = {"hardware": "AMD Instinct MI355X (1 GPU)", "reference_hardware": pub["hardware"],
              "cpu": cpu,
              "rule": "best bsmr_gflops over alpha x delta (analyze_results.cpp:283-345), "
                      "10 back-to-back launches per setting (warm, as the reference)",
              "matrices": {}}
    for name in args.matrices.split(","):
        M, N, rp, ci = synth.SUITESPARSE_REBUILDS[name]()
        path = os.path.join(args.out, f"{name}.mtx")
        t0 = time.time()
        synth.write_mtx(path, M, N, rp, ci)
        logdir = os.path.join(args.out, f"logs_{name}") + "/"
        os.makedirs(logdir, exist_ok=True)
        t1 = time.time()
        r = subprocess.run([BIN, "-f", path, "-t", "1", "-l", logdir], capture_output=True,
                           text=True, timeout=1500)
        if r.returncode != 0:
            raise SystemExit(f"{name}: BSMR-sddmm failed: {r.stderr[-2000:]}")
        t2 = time.time()
        if not args.keep_mtx:
            os.remove(path)
        logs = parse_logs(logdir)
        per_k = {}
        for K in (32, 64, 128, 256):
            cand = {(a, d): v for (k, a, d), v in logs.items() if k == K}
            (a, d), (gf, ms) = max(cand.items(), key=lambda kv: kv[1][0])
            ref = published.get((name, K), {})
            per_k[str(K)] = {
                "mi355x_gflops": gf, "mi355x_sddmm_ms": ms, "alpha": a, "delta": d,
                "rtx4090_bsmr_gflops": ref.get("BSMR"), "rtx4090_cusparse_gflops": ref.get("cuSPARSE"),
                "rtx4090_best_any_gflops": max((ref.get(c, 0.0) for c in (
                    "BSMR", "cuSDDMM", "cuSPARSE", "RoDe", "ASpT", "TCGNN", "FlashSparse",
                    "Sputnik")), default=None) if ref else None,
                "speedup_vs_rtx4090_bsmr": round(gf / ref["BSMR"], 2) if ref else None,
                "published_source": ref.get("source"),
                "settings_measured": len(cand),
            }
        entry = {"M": M, "N": N, "nnz": len(ci), "write_mtx_s": round(t1 - t0, 1),
                 "test_mode_s": round(t2 - t1, 1), "K": per_k}
        if not args.no_k512:
            entry["K"]["512"] = k512(name, M, N, rp, ci)
        for K, v in entry["K"].items():
            v.update(retime_and_cpu(M, N, rp, ci, int(K), v["alpha"], v["delta"]))
        result["matrices"][name] = entry
        print(json.dumps({name: {k: (v["mi355x_gflops"] if "mi355x_gflops" in v else v["gflops"])
                                 for k, v in entry["K"].items()}}), flush=True)
    with open(os.path.join(args.out, "compare.json"), "w") as f:
        json.dump(result, f, indent=1)
    print(json.dumps(result))


if __name__ == "__main__":
    main()
