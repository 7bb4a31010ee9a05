#!/bin/bash
# 2 KiB-row rule restricted to non-sparse rows: GPU suite + SuiteSparse comparison (final tree).
set -o pipefail
OUT=gpurun_out/r03w
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*" >> "$OUT/steps.log"; }
step pytest && timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
step smoke && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
step suitesparse && timeout -k 10 900 python3 -u tools/suitesparse_compare.py --out "$OUT/ss" > "$OUT/ss.log" 2>&1
rc=$?
step "done rc=$rc"
exit $rc
