#!/bin/bash
# L2-miss traffic of the C4 x1 launch with and without row-block pairs: FETCH_SIZE, WRITE_SIZE and
# TCC hit / miss (separate rocprofv3 passes) of tools/prof_sddmm.py at BSMR_DIAG 0 (pairs) and
# 16384 (pairs off). Through gpurun:  bash tools/gpu_pairs_traffic.sh <tag> [scale]
set -o pipefail
TAG=${1:-pairs_traffic}; SCALE=${2:-1.0}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # $1 = name, $2 = diag, rest = counters
    local name=$1 diag=$2; shift 2
    echo "[$(date +%T)] $name" >> "$OUT/steps.log"
    timeout -s KILL 300 rocprofv3 --pmc "$@" --kernel-include-regex k_sddmm --output-format csv \
        -d "$OUT/$name" -o run -- python3 tools/prof_sddmm.py --iters 3 --workload reddit_like \
        --scale "$SCALE" --diag "$diag" > "$OUT/$name.log" 2>&1
}
for d in 0 16384; do
    run fetch_$d $d FETCH_SIZE && run write_$d $d WRITE_SIZE && run tcc_$d $d TCC_HIT_sum TCC_MISS_sum || exit $?
done
for d in 0 16384; do
    mkdir -p "$OUT/all_$d" && for k in fetch write tcc; do cp -r "$OUT/${k}_$d" "$OUT/all_$d/"; done
    python3 tools/pmc_table.py "$OUT/all_$d" > "$OUT/table_$d.json" || exit $?
done
echo done >> "$OUT/steps.log"
