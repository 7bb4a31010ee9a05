#!/bin/bash
# A/B timing of several BSMR_* settings on one ab_env.sh config (through gpurun):
#   bash tools/ab_grid.sh <tag> <config> "VAR=v,VAR2=w" "VAR=x" ...   ("-" = no setting)
# Each setting runs tools/prof_sddmm.py once; summary.txt gets one line per setting.
set -o pipefail
TAG=$1; CFG=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
case "$CFG" in
    C2) ARGS="--workload nips_like --K 128 --dtype f32" ;;
    C3) ARGS="--workload cop20k_like --K 256 --dtype f16" ;;
    C4) ARGS="--workload reddit_like --scale 0.5 --K 128 --dtype f32" ;;
    C4x1) ARGS="--workload reddit_like --scale 1.0 --K 128 --dtype f32" ;;
    C5u) ARGS="--workload dlmc_like --mask uniform --K 512 --dtype bf16" ;;
    M15k64) ARGS="--workload mycielskian15 --K 64 --alpha 0.3 --delta 0.1" ;;
    M16k128) ARGS="--workload mycielskian16 --K 128 --alpha 0.3 --delta 0.1" ;;
    M14k128) ARGS="--workload mycielskian14 --K 128 --alpha 0.5 --delta 0.3" ;;
    M15k256) ARGS="--workload mycielskian15 --K 256 --alpha 0.5 --delta 0.7" ;;
    M16k256) ARGS="--workload mycielskian16 --K 256 --alpha 0.5 --delta 0.7" ;;
    M16k512) ARGS="--workload mycielskian16 --K 512 --alpha 0.5 --delta 0.5" ;;
    M16k64) ARGS="--workload mycielskian16 --K 64 --alpha 0.3 --delta 0.1" ;;
    M15k128) ARGS="--workload mycielskian15 --K 128 --alpha 0.7 --delta 0.3" ;;
    T128) ARGS="--workload Trefethen_20000 --K 128 --alpha 0.7 --delta 0.5" ;;
    *) echo "unknown config $CFG" >&2; exit 2 ;;
esac
n=0
for set in "$@"; do
    n=$((n + 1))
    envs=""; [ "$set" != "-" ] && envs="BSMR_${set//,/ BSMR_}"
    env $envs timeout -k 10 300 python3 tools/prof_sddmm.py --iters 50 $ARGS > "$OUT/${CFG}_$n.json" 2> "$OUT/${CFG}_$n.err" || exit $?
    echo "$CFG [$set] $(python3 -c "import json; d=json.loads(open('$OUT/${CFG}_$n.json').read().strip().splitlines()[-1]); print(d['timing_ms'])")" | tee -a "$OUT/summary.txt"
done
