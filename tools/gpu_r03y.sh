#!/bin/bash
# C4 x1 column-range A/B, three alternating repetitions (staged 4 MiB default vs 8 MiB).
set -o pipefail
OUT=gpurun_out/r03y
mkdir -p "$OUT"
export TMPDIR=/tmp
Q="--no-cpu-baseline --no-vendor --pmc off --cold-steps 0 --steps 20 --warmup 3"
for rep in 1 2 3; do
  for v in def 8192; do
    if [ $v = def ]; then E=""; else E="BSMR_L2_RANGE_KB=$v"; fi
    env $E timeout -k 10 400 python3 bench.py --config C4 --scale 1.0 $Q > "$OUT/c4_${v}_r$rep.json" 2> "$OUT/c4_${v}_r$rep.err" || exit 1
  done
done
