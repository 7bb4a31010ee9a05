#!/bin/bash
# Item cost calibration: per-item timelines (tools/item_trace.py) over row-block sizes and
# workloads. Through gpurun: bash tools/gpu_itemcal.sh <tag>
set -o pipefail
TAG=${1:-itemcal}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {  # name, env, args
    local name=$1 envs=$2; shift 2
    env $envs timeout -k 10 150 python3 tools/item_trace.py --out "$OUT/$name" "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || return $?
    echo "$name $envs $(tail -n 1 $OUT/$name.json)" >> "$OUT/summary.txt"
}
for K in 256 512; do
    for rb in 0 32 48 80 112; do
        e="BSMR_RB_ROWS=$rb"; [ $rb = 0 ] && e="BSMR_DIAG=0"
        [ $K = 512 ] && [ $rb = 112 ] && continue
        run "myc15_K${K}_rb$rb" "$e" --workload mycielskian15 --K $K --alpha 0.5 --delta 0.7 || exit $?
        run "myc16_K${K}_rb$rb" "$e" --workload mycielskian16 --K $K --alpha 0.5 --delta 0.7 || exit $?
    done
done
for K in 64 128; do
    for rb in 0 16 32 48 96; do
        e="BSMR_RB_ROWS=$rb"; [ $rb = 0 ] && e="BSMR_DIAG=0"
        run "tref_K${K}_rb$rb" "$e" --workload Trefethen_20000 --K $K --alpha 0.1 --delta 0.5 || exit $?
    done
done
run C2 "BSMR_DIAG=0" --workload nips_like --K 128 || exit $?
run C3 "BSMR_DIAG=0" --workload cop20k_like --K 256 --dtype f16 || exit $?
run C4q "BSMR_DIAG=0" --workload reddit_like --scale 0.25 --K 128 || exit $?
run myc14_K128 "BSMR_DIAG=0" --workload mycielskian14 --K 128 --alpha 0.3 --delta 0.3 || exit $?
echo done >> "$OUT/summary.txt"
