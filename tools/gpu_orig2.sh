#!/bin/bash
# C3 with original-order row blocks dealt round-robin (default) or contiguously per XCD
# (BSMR_ORIG_CONTIG=1). Usage (through gpurun): bash tools/gpu_orig2.sh <tag>
set -o pipefail
O=gpurun_out/${1:-orig2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -x -q -m gpu -k "original_order" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for r in 1 2; do for v in 0 1; do
  BSMR_ORIG_CONTIG=$v timeout -k 10 300 python3 bench.py --config C3 --steps 50 --warmup 5 --no-cpu-baseline --no-vendor --cold-steps 0 --no-split > $O/C3_c${v}_$r.json 2>> $O/err.log || exit 1
done; done
