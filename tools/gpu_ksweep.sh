#!/bin/bash
# K-anomaly sweep on the rebuilt SuiteSparse matrices: rows per row block
# (BSMR_RB_ROWS), one item per segment and the column-major launch, at the K points where the
# published-comparison anomalies sit. Through gpurun: bash tools/gpu_ksweep.sh <tag>
set -o pipefail
TAG=${1:-ksweep}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {  # name, env, args
    local name=$1 envs=$2; shift 2
    env $envs timeout -k 10 120 python3 tools/prof_sddmm.py --iters 50 "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || return $?
    echo "$name $envs $* $(python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print(d['timing_ms']['total_ms'], d['rb'])")" >> "$OUT/summary.txt"
}
for K in 32 64 128 256; do
    for rb in 0 16 32 48 64 96 128; do
        e="BSMR_RB_ROWS=$rb"; [ $rb = 0 ] && e="BSMR_DIAG=0"
        run "tref_K${K}_rb$rb" "$e" --workload Trefethen_20000 --K $K --alpha 0.1 --delta 0.0 || exit $?
    done
    run "tref_K${K}_cm" "BSMR_DIAG=0" --workload Trefethen_20000 --K $K --alpha 0.1 --delta 0.0 --layout colmajor || exit $?
done
for m in mycielskian15 mycielskian16; do
    for K in 256 512; do
        for rb in 0 32 48 80; do
            e="BSMR_RB_ROWS=$rb"; [ $rb = 0 ] && e="BSMR_DIAG=0"
            run "${m}_K${K}_rb$rb" "$e" --workload $m --K $K --alpha 0.5 --delta 0.7 || exit $?
        done
        run "${m}_K${K}_cm" "BSMR_DIAG=0" --workload $m --K $K --alpha 0.5 --delta 0.7 --layout colmajor || exit $?
    done
done
echo done >> "$OUT/summary.txt"
