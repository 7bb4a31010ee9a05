#!/bin/bash
# Clustering check + timing through gpurun: plan bit-exactness / reference-log tests, then plan
# build times of reddit-like x0.25 / x0.5 / x1.
#   bash tools/gpu_cluster.sh <tag> [scales]
set -o pipefail
O=gpurun_out/${1:-cluster}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu -k "plan or exact or cluster or import_rows" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 &&
for s in ${2:-0.25 0.5}; do
  timeout -k 10 400 python3 tools/plan_time.py --workload reddit_like --scale $s --batches 16384 > $O/plan_c4_$s.json 2>> $O/err.log || exit 1
done
