#!/bin/bash
# A/B timing of one environment switch on the bench configs (through gpurun):
#   bash tools/ab_env.sh <tag> VAR[,VAR2...] "valA valB" [configs]   (every VAR set to the value)
set -o pipefail
TAG=$1; VAR=$2; VALS=$3; CFGS=${4:-"C2 C4 C3"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for c in $CFGS; do
    case "$c" in
        C2) ARGS="--workload nips_like --K 128 --dtype f32" ;;
        C2k32) ARGS="--workload nips_like --K 32 --dtype f32" ;;
        C2k64) ARGS="--workload nips_like --K 64 --dtype f32" ;;
        C2k256) ARGS="--workload nips_like --K 256 --dtype f32" ;;
        C2k512) ARGS="--workload nips_like --K 512 --dtype f32" ;;
        C3) ARGS="--workload cop20k_like --K 256 --dtype f16" ;;
        C4) ARGS="--workload reddit_like --scale 0.5 --K 128 --dtype f32" ;;
        C4x1) ARGS="--workload reddit_like --scale 1.0 --K 128 --dtype f32" ;;
        C5u) ARGS="--workload dlmc_like --mask uniform --K 512 --dtype bf16" ;;
        C5b) ARGS="--workload dlmc_like --mask block --K 512 --dtype bf16" ;;
        M14) ARGS="--workload mycielskian14 --K 128 --alpha 0.3 --delta 0.3" ;;
        M15) ARGS="--workload mycielskian15 --K 256 --alpha 0.5 --delta 0.7" ;;
        M15k512) ARGS="--workload mycielskian15 --K 512 --alpha 0.5 --delta 0.7" ;;
        M16) ARGS="--workload mycielskian16 --K 256 --alpha 0.5 --delta 0.7" ;;
        M16k512) ARGS="--workload mycielskian16 --K 512 --alpha 0.5 --delta 0.7" ;;
        T64) ARGS="--workload Trefethen_20000 --K 64 --alpha 0.1 --delta 0.5" ;;
        T128) ARGS="--workload Trefethen_20000 --K 128 --alpha 0.1 --delta 0.5" ;;
        M15k32) ARGS="--workload mycielskian15 --K 32 --alpha 0.9 --delta 0.1" ;;
        M15k64) ARGS="--workload mycielskian15 --K 64 --alpha 0.3 --delta 0.1" ;;
    esac
    for v in $VALS; do
        sets=""; for V in ${VAR//,/ }; do sets="$sets $V=$v"; done
        env $sets timeout -k 10 300 python3 tools/prof_sddmm.py --iters 50 $ARGS > "$OUT/${c}_$v.json" 2> "$OUT/${c}_$v.err" || exit $?
        echo "$c $VAR=$v $(python3 -c "import json,sys; d=json.loads(open('$OUT/${c}_$v.json').read().strip().splitlines()[-1]); print(d['timing_ms'])")" | tee -a "$OUT/summary.txt"
    done
done
