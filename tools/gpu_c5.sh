#!/bin/bash
set -o pipefail
TAG=${1:-c5}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q > "$OUT/pytest.log" 2>&1 || exit 1
for m in uniform block; do
  for L in auto; do
    timeout -k 10 120 python3 bench.py --config C5 --mask $m --steps 100 --warmup 10 --no-cpu-baseline --cold-steps 0 --layout $L > "$OUT/c5_${m}_$L.json" 2>>"$OUT/err.log" || exit 1
  done
done
