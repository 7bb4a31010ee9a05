#!/bin/bash
# Wave stall counters of one config's SDDMM launch (through gpurun): two SQ passes, each a run of
# its own, over tools/prof_sddmm.py; with STAGE_ONLY=1 also the staging-only ablation (BSMR_DIAG=8)
# so the piece phase can be taken as the difference.
#   bash tools/gpu_stall_pmc.sh <tag> <C2|C3|C4>
set -o pipefail
TAG=${1:-stall}; CFG=${2:-C2}
OUT=gpurun_out/$TAG/$CFG
mkdir -p "$OUT"
export TMPDIR=/tmp
case "$CFG" in
    C2) ARGS="--workload nips_like --K 128 --dtype f32" ;;
    C3) ARGS="--workload cop20k_like --K 256 --dtype f16" ;;
    C4) ARGS="--workload reddit_like --scale 0.5 --K 128 --dtype f32" ;;
    *) echo "unknown config $CFG"; exit 2 ;;
esac
run() {  # $1 = name, rest = counters
    local name=$1; shift
    timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-include-regex k_sddmm --output-format csv \
        -d "$OUT/$name" -o run -- python3 tools/prof_sddmm.py --iters 10 $ARGS > "$OUT/$name.log" 2>&1
}
run wait SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS &&
run inst SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH \
    SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES &&
if [ "${STAGE_ONLY:-0}" = 1 ]; then
    BSMR_DIAG=8 run wait_stage SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS \
        SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
fi
