#!/bin/bash
# A/B timing of one environment switch on the bench configs (through gpurun):
#   bash tools/ab_env.sh <tag> VAR "valA valB" [configs]
set -o pipefail
TAG=$1; VAR=$2; VALS=$3; CFGS=${4:-"C2 C4 C3"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for c in $CFGS; do
    case "$c" in
        C2) ARGS="--workload nips_like --K 128 --dtype f32" ;;
        C3) ARGS="--workload cop20k_like --K 256 --dtype f16" ;;
        C4) ARGS="--workload reddit_like --scale 0.5 --K 128 --dtype f32" ;;
        C4x1) ARGS="--workload reddit_like --scale 1.0 --K 128 --dtype f32" ;;
        C5u) ARGS="--workload dlmc_like --mask uniform --K 512 --dtype bf16" ;;
        C5b) ARGS="--workload dlmc_like --mask block --K 512 --dtype bf16" ;;
    esac
    for v in $VALS; do
        env "$VAR=$v" timeout -k 10 300 python3 tools/prof_sddmm.py --iters 50 $ARGS > "$OUT/${c}_$v.json" 2> "$OUT/${c}_$v.err" || exit $?
        echo "$c $VAR=$v $(python3 -c "import json,sys; d=json.loads(open('$OUT/${c}_$v.json').read().strip().splitlines()[-1]); print(d['timing_ms'])")" | tee -a "$OUT/summary.txt"
    done
done
