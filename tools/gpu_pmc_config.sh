#!/bin/bash
# Counter evidence for one BASELINE config (through gpurun): a rocprofv3 kernel-trace summary and
# separate PMC passes (one counter group per run, kernel-trace only) over tools/prof_sddmm.py:
# FETCH_SIZE, WRITE_SIZE, L2 hit/miss, MFMA busy + MFMA op counts, LDS/VALU activity.
#   bash tools/gpu_pmc_config.sh <tag> <C2|C3|C4|C5u|C5b>
set -o pipefail
TAG=${1:-pmc}
CFG=${2:-C2}
OUT=gpurun_out/$TAG/$CFG
mkdir -p "$OUT"
export TMPDIR=/tmp
case "$CFG" in
    C2) ARGS="--workload nips_like --K 128 --dtype f32" ;;
    C3) ARGS="--workload cop20k_like --K 256 --dtype f16" ;;
    C4) ARGS="--workload reddit_like --scale 0.5 --K 128 --dtype f32" ;;
    C5u) ARGS="--workload dlmc_like --mask uniform --K 512 --dtype bf16" ;;
    C5b) ARGS="--workload dlmc_like --mask block --K 512 --dtype bf16" ;;
    *) echo "unknown config $CFG"; exit 2 ;;
esac
ITERS=${ITERS:-10}
run() {  # $1 = name, rest = counters
    local name=$1; shift
    timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-include-regex k_sddmm --output-format csv \
        -d "$OUT/$name" -o run -- python3 tools/prof_sddmm.py --iters "$ITERS" $ARGS \
        > "$OUT/$name.log" 2>&1
}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 tools/prof_sddmm.py --iters "$ITERS" $ARGS > "$OUT/trace.log" 2>&1 &&
run fetch FETCH_SIZE &&
run write WRITE_SIZE &&
run tcc TCC_HIT_sum TCC_MISS_sum &&
run mfma SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 \
    SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_MFMA GRBM_GUI_ACTIVE &&
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS \
    SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY
rc=$?
echo "rc=$rc" > "$OUT/rc.txt"
exit $rc
