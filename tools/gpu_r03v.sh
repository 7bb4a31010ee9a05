#!/bin/bash
# 2 KiB-row layout rule: GPU suite, K = 512 / 256 defaults on the mycielskian rebuilds, then the
# SuiteSparse comparison on the final tree.
set -o pipefail
OUT=gpurun_out/r03v
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*" >> "$OUT/steps.log"; }
run() { timeout -k 10 300 python3 tools/rb_sweep.py "$@" --set "" >> "$OUT/sweep.jsonl" 2>> "$OUT/sweep.err"; }
step pytest && timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
step sweep && run --workload mycielskian14 --K 512 --alpha 0.5 --delta 0.7 &&
run --workload mycielskian15 --K 512 --alpha 0.5 --delta 0.3 &&
run --workload mycielskian16 --K 512 --alpha 0.5 --delta 0.7 &&
run --workload mycielskian14 --K 256 --alpha 0.5 --delta 0.3 &&
run --workload mycielskian15 --K 256 --alpha 0.3 --delta 0.1 &&
run --workload mycielskian16 --K 256 --alpha 0.5 --delta 1.1 &&
step suitesparse && timeout -k 10 900 python3 -u tools/suitesparse_compare.py --out "$OUT/ss" > "$OUT/ss.log" 2>&1
rc=$?
step "done rc=$rc"
exit $rc
