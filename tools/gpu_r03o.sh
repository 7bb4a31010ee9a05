#!/bin/bash
# Split-K dense-sampled launch: parity tests, then C5 uniform / block A/B (BSMR_DENSE_SPLIT 1 vs 2).
set -o pipefail
OUT=gpurun_out/r03o
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*" >> "$OUT/steps.log"; }
Q="--no-cpu-baseline --no-vendor --pmc off --cold-steps 0 --steps 200 --warmup 20"
step tests && timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dtypes_cli.py -x -v -m gpu -k "dense" --timeout 300 --timeout-method thread > "$OUT/pytest_dense.log" 2>&1 &&
for rep in 1 2; do
  for sp in 1 2; do
    for mask in uniform block; do
      step "C5 $mask split $sp rep $rep" && BSMR_DENSE_SPLIT=$sp timeout -k 10 300 python3 bench.py --config C5 --mask $mask $Q > "$OUT/c5_${mask}_s${sp}_r${rep}.json" 2> "$OUT/c5_${mask}_s${sp}_r${rep}.err" || exit 1
    done
  done
done
step K256 && BSMR_DENSE_SPLIT=2 timeout -k 10 300 python3 bench.py --config C5 --K 256 $Q > "$OUT/c5_uniform_s2_k256.json" 2> "$OUT/c5_k256.err"
rc=$?
step "done rc=$rc"
exit $rc
