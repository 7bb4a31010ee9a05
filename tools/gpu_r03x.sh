#!/bin/bash
# Column-range size A/B beyond the current rules: 2 KiB rows at 16 / 32 MiB, C4 x1 and C3
# (512-byte rows, staged) at 6 / 8 MiB.
set -o pipefail
OUT=gpurun_out/r03x
mkdir -p "$OUT"
export TMPDIR=/tmp
Q="--no-cpu-baseline --no-vendor --pmc off --cold-steps 0"
timeout -k 10 300 python3 tools/rb_sweep.py --workload mycielskian16 --K 512 --alpha 0.5 --delta 0.7 --set "" --set BSMR_L2_RANGE_KB=16384 --set BSMR_L2_RANGE_KB=32768 >> "$OUT/sweep.jsonl" 2>> "$OUT/sweep.err" &&
timeout -k 10 300 python3 tools/rb_sweep.py --workload mycielskian15 --K 512 --alpha 0.5 --delta 0.3 --set "" --set BSMR_L2_RANGE_KB=16384 >> "$OUT/sweep.jsonl" 2>> "$OUT/sweep.err" &&
for v in def 8192 6144; do
  if [ $v = def ]; then E=""; else E="BSMR_L2_RANGE_KB=$v"; fi
  env $E timeout -k 10 400 python3 bench.py --config C4 --scale 1.0 --steps 10 --warmup 2 $Q > "$OUT/c4_$v.json" 2> "$OUT/c4_$v.err" || exit 1
done &&
for v in def 8192; do
  if [ $v = def ]; then E=""; else E="BSMR_L2_RANGE_KB=$v"; fi
  env $E timeout -k 10 300 python3 bench.py --config C3 --steps 50 --warmup 5 $Q > "$OUT/c3_$v.json" 2> "$OUT/c3_$v.err" || exit 1
done
