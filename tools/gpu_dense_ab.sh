#!/bin/bash
# Dense-sampled launch A/B after a kernel change (through gpurun): the dense GPU tests, then the
# C5 uniform / block bench lines twice each (no PMC, CPU or vendor legs).
#   bash tools/gpu_dense_ab.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-dense_ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -x -q -m gpu -k "dense or C5 or dlmc" --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 &&
for i in 1 2; do
    for m in uniform block; do
        timeout -k 10 120 python3 bench.py --config C5 --mask $m --steps 200 --warmup 20 --no-cpu-baseline --no-vendor --pmc off > "$OUT/c5_${m}_$i.json" 2> "$OUT/c5_${m}_$i.err" || exit $?
    done
done
