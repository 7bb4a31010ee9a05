#!/bin/bash
# Round-3 re-entry check: smoke + GPU suite on the rebuilt tree, then C5 uniform at K = 256 / 512
# (k-loop scaling of the dense-sampled launch) and C2 quick line.
set -o pipefail
OUT=gpurun_out/r03n
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*" >> "$OUT/steps.log"; }
Q="--no-cpu-baseline --no-vendor --pmc off --cold-steps 0"
step smoke && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
step pytest && timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
step C5u512 && timeout -k 10 300 python3 bench.py --config C5 --steps 200 --warmup 20 $Q > "$OUT/c5u_512.json" 2> "$OUT/c5u_512.err" &&
step C5u256 && timeout -k 10 300 python3 bench.py --config C5 --K 256 --steps 200 --warmup 20 $Q > "$OUT/c5u_256.json" 2> "$OUT/c5u_256.err" &&
step C5u128 && timeout -k 10 300 python3 bench.py --config C5 --K 128 --steps 200 --warmup 20 $Q > "$OUT/c5u_128.json" 2> "$OUT/c5u_128.err" &&
step C2 && timeout -k 10 300 python3 bench.py $Q > "$OUT/c2.json" 2> "$OUT/c2.err"
rc=$?
step "done rc=$rc"
exit $rc
