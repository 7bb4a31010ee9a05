#!/bin/bash
# Original-order row blocks (BSMR_ORIG_ROWS): layout GPU tests, then C3 / C2 bench lines with
# the switch off, auto and forced. Usage (through gpurun): bash tools/gpu_orig.sh <tag>
set -o pipefail
O=gpurun_out/${1:-orig}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -x -q -m gpu -k "layout_variants or original_order or shard" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for v in 0 auto 1; do
  BSMR_ORIG_ROWS=$v timeout -k 10 300 python3 bench.py --config C3 --steps 50 --warmup 5 --no-cpu-baseline --no-vendor --cold-steps 0 --no-split > $O/C3_$v.json 2>> $O/err.log || exit 1
done
for v in 0 1; do
  BSMR_ORIG_ROWS=$v timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-vendor --cold-steps 0 --no-split > $O/C2_$v.json 2>> $O/err.log || exit 1
done
