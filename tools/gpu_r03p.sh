#!/bin/bash
# Packed output (CSR position in the metadata word): parity tests, then C2 A/B (BSMR_OUT_PACKED
# 1 vs 0, three alternating repetitions) and one packed C2 line with in-run PMC traffic.
set -o pipefail
OUT=gpurun_out/r03p
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*" >> "$OUT/steps.log"; }
Q="--no-cpu-baseline --no-vendor --pmc off --cold-steps 0 --steps 400 --warmup 40"
step tests && timeout -k 10 900 python3 -u -m pytest tests/test_gpu_out_packed.py tests/test_gpu_parity.py tests/test_gpu_item_sched.py -x -v -m gpu --timeout 600 --timeout-method thread > "$OUT/pytest.log" 2>&1 &&
for rep in 1 2 3; do
  for pk in 1 0; do
    step "C2 packed $pk rep $rep" && BSMR_OUT_PACKED=$pk timeout -k 10 300 python3 bench.py $Q > "$OUT/c2_p${pk}_r${rep}.json" 2> "$OUT/c2_p${pk}_r${rep}.err" || exit 1
  done
done
step C2pmc && timeout -k 10 300 python3 bench.py --no-vendor --cold-steps 0 > "$OUT/c2_pmc.json" 2> "$OUT/c2_pmc.err"
rc=$?
step "done rc=$rc"
exit $rc
