#!/bin/bash
# PMC passes over the SDDMM kernel (one counter group per rocprofv3 run, kernel-trace only, no
# sys/runtime tracing). Usage through gpurun: bash tools/gpu_pmc.sh <tag> [K]
set -o pipefail
TAG=${1:-pmc}
K=${2:-128}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # $1 = name, rest = counters
    local name=$1; shift
    timeout -k 10 240 rocprofv3 --pmc "$@" --kernel-include-regex k_sddmm --output-format csv \
        -d "$OUT/$name" -o run -- python3 tools/prof_sddmm.py --iters 10 --K "$K" \
        > "$OUT/$name.log" 2>&1
}
timeout -k 10 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1
run fetch FETCH_SIZE &&
run write WRITE_SIZE &&
run tcc TCC_HIT_sum TCC_MISS_sum &&
run ta TA_TA_BUSY_sum TA_BUSY_avr GRBM_GUI_ACTIVE &&
run sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 tools/prof_sddmm.py --iters 10 --K "$K" > "$OUT/trace.log" 2>&1
rc=$?
echo "rc=$rc" > "$OUT/rc.txt"
exit $rc
