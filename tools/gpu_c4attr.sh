#!/bin/bash
# Attribution of the C4 row-block launch's L2-miss (HBM + Infinity Cache) traffic by stream:
# FETCH_SIZE of the full launch and of three ablations (BSMR_DIAG, sddmm.hip: 8 = staging only,
# 64 = every piece reads B column 0 so B gathers hit L2, 128 = no P stores), WRITE_SIZE and the
# L2 hit rate of the full launch. Through gpurun:
#   bash tools/gpu_c4attr.sh <tag> [scale] [extra prof_sddmm args]
set -o pipefail
TAG=${1:-c4attr}
SCALE=${2:-1.0}
shift 2
EXTRA="$*"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # $1 = name, $2 = diag, rest = counters
    local name=$1 diag=$2; shift 2
    echo "[$(date +%T)] $name" >> "$OUT/steps.log"
    timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex k_sddmm --output-format csv \
        -d "$OUT/$name" -o run -- python3 tools/prof_sddmm.py --iters 3 --workload reddit_like \
        --scale "$SCALE" --diag "$diag" $EXTRA > "$OUT/$name.log" 2>&1
}
run trace_fetch 0 FETCH_SIZE &&
run write 0 WRITE_SIZE &&
run tcc 0 TCC_HIT_sum TCC_MISS_sum &&
run fetch_stage 8 FETCH_SIZE &&
run fetch_bl2 64 FETCH_SIZE &&
run fetch_nostore 128 FETCH_SIZE
rc=$?
echo "rc=$rc" > "$OUT/rc.txt"
exit $rc
