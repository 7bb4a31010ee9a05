#!/bin/bash
# LDS / VALU counter passes over the C2 row-block launch (tools/prof_sddmm.py): bank conflicts
# vs LDS-array cycles, LDS instruction counts and waits, VALU activity. Through gpurun:
#   bash tools/gpu_ldspmc.sh <tag>
set -o pipefail
O=gpurun_out/${1:-ldspmc}
mkdir -p $O
export TMPDIR=/tmp
run() {
    local name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex k_sddmm --output-format csv \
        -d "$O/$name" -o run -- python3 tools/prof_sddmm.py --iters 10 > "$O/$name.log" 2>&1
}
run lds1 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS &&
run lds2 SQ_ACTIVE_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL &&
run valu SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES
