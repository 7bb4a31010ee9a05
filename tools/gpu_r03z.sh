#!/bin/bash
# Validation of the 8 MiB staged 512-byte-row ranges: GPU suite + smoke, C4 x1 and C3 bench lines
# with in-run PMC traffic.
set -o pipefail
OUT=gpurun_out/r03z
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*" >> "$OUT/steps.log"; }
step pytest && timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
step smoke && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
step C4 && timeout -k 10 600 python3 bench.py --config C4 --scale 1.0 --steps 20 --warmup 3 --cold-steps 0 > "$OUT/bench_C4x1.json" 2> "$OUT/bench_C4x1.err" &&
step C3 && timeout -k 10 600 python3 bench.py --config C3 --steps 50 --warmup 5 > "$OUT/bench_C3.json" 2> "$OUT/bench_C3.err"
rc=$?
step "done rc=$rc"
exit $rc
