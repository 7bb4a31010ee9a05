#!/bin/bash
# Bench lines for the other BASELINE.json configs (through gpurun): bash tools/gpu_configs.sh <tag> [c4scale]
set -o pipefail
TAG=${1:-cfg}
S4=${2:-0.25}
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config C3 --steps 100 > "$OUT/bench_C3_$TAG.json" 2> "$OUT/bench_C3_$TAG.err" &&
timeout -k 10 300 python bench.py --config C5 --mask uniform --steps 100 > "$OUT/bench_C5u_$TAG.json" 2> "$OUT/bench_C5u_$TAG.err" &&
timeout -k 10 300 python bench.py --config C5 --mask block --steps 100 > "$OUT/bench_C5b_$TAG.json" 2> "$OUT/bench_C5b_$TAG.err" &&
timeout -k 10 600 python bench.py --config C4 --scale "$S4" --steps 50 > "$OUT/bench_C4_$TAG.json" 2> "$OUT/bench_C4_$TAG.err"
rc=$?
echo "rc=$rc" > "$OUT/configs_$TAG.rc"
exit $rc
