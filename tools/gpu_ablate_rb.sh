#!/bin/bash
# Row-block kernel ablations on one config (profiling only; results are wrong under BSMR_DIAG):
# 0 real, 8 staging only, 64 B gathers hit column 0, 128 no P stores (staged output), 192 both.
#   bash tools/gpu_ablate_rb.sh <tag> <C2|C3|C4>
set -o pipefail
TAG=${1:-ablrb}; CFG=${2:-C4}
OUT=gpurun_out/$TAG/$CFG
mkdir -p "$OUT"
case "$CFG" in
    C2) ARGS="--workload nips_like --K 128 --dtype f32" ;;
    C3) ARGS="--workload cop20k_like --K 256 --dtype f16" ;;
    C4) ARGS="--workload reddit_like --scale 0.5 --K 128 --dtype f32" ;;
esac
for d in 0 8 64 128 192; do
    timeout -k 10 300 python3 tools/prof_sddmm.py --iters 30 --diag $d $ARGS > "$OUT/diag_$d.json" 2> "$OUT/diag_$d.err" || exit $?
    echo "$CFG diag=$d $(python3 -c "import json; d=json.loads(open('$OUT/diag_$d.json').read().strip().splitlines()[-1]); print(d['timing_ms']['total_ms'])")" | tee -a "$OUT/summary.txt"
done
