#!/bin/bash
# Ablation timings of the SDDMM kernel (profiling only; results are wrong under BSMR_DIAG):
# 0 = real, 1 = no P stores, 2 = A gathers hit one row, 4 = B gathers hit one column, 7 = all.
set -o pipefail
TAG=${1:-abl}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ok=0
for d in 0 1 2 4 6 7; do
    BSMR_DIAG=$d timeout -k 10 120 python3 tools/prof_sddmm.py --iters 50 > "$OUT/diag_$d.json" 2>> "$OUT/err.log" || { ok=1; break; }
done
echo "rc=$ok" > "$OUT/rc.txt"
exit $ok
