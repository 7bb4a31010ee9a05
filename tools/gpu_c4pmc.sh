#!/bin/bash
# C4 (reddit-like, x SCALE) counter passes over the row-block SDDMM kernel: HBM/MALL bytes, L2
# hit rate, TA busy, SQ wait/VMEM counts; then a kernel-trace summary. Through gpurun:
#   bash tools/gpu_c4pmc.sh <tag> [scale] [extra prof_sddmm args]
set -o pipefail
TAG=${1:-c4pmc}
SCALE=${2:-0.25}
shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # $1 = name, rest = counters
    local name=$1; shift
    timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex k_sddmm --output-format csv \
        -d "$OUT/$name" -o run -- python3 tools/prof_sddmm.py --iters 3 --workload reddit_like \
        --scale "$SCALE" $EXTRA > "$OUT/$name.log" 2>&1
}
EXTRA="$*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 tools/prof_sddmm.py --iters 3 --workload reddit_like --scale "$SCALE" $EXTRA > "$OUT/trace.log" 2>&1 &&
run fetch FETCH_SIZE &&
run tcc TCC_HIT_sum TCC_MISS_sum &&
run ta TA_TA_BUSY_sum TA_BUSY_avr GRBM_GUI_ACTIVE &&
run sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY
rc=$?
echo "rc=$rc" > "$OUT/rc.txt"
exit $rc
