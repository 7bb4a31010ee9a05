#!/bin/bash
# Plan-build (clustering) A/B of library variants on reddit-like: the in-tree build and each
# sddmm-gpu_amd/lib_<variant>/libbsmr_amd.so, the same permutation required (rows sha256).
#   bash tools/gpu_plan_ab.sh <tag> <scale> "variant1 variant2 ..."
set -o pipefail
TAG=$1; SCALE=${2:-0.5}; VARS=${3:-""}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python3 tools/plan_time.py --workload reddit_like --scale "$SCALE" --batches 16384 > "$OUT/plan_intree_$SCALE.json" 2> "$OUT/plan_intree_$SCALE.err" || exit $?
for v in $VARS; do
    BSMR_LIB_PATH=$GRAFT_REPO_ROOT/sddmm-gpu_amd/lib_$v/libbsmr_amd.so timeout -k 10 300 python3 tools/plan_time.py --workload reddit_like --scale "$SCALE" --batches 16384 > "$OUT/plan_${v}_$SCALE.json" 2> "$OUT/plan_${v}_$SCALE.err" || exit $?
done
for f in "$OUT"/plan_*_"$SCALE".json; do
    python3 -c "import json,sys; d=json.load(open('$f')); r=list(d['runs'].values())[0]; print('$f', r['row_reorder_ms'], r['rows_sha256'], r['num_clusters'])" | tee -a "$OUT/summary.txt"
done
