#!/bin/bash
# C4 (reddit-like x0.5, fp32 K=128) layout sweep: L2 column-range budget x LDS budget (through
# gpurun): bash tools/sweep_c4.sh <tag> "<l2 kb list>" "<lds kb list>" [scale]
set -o pipefail
TAG=$1; L2S=$2; LDSS=$3; SCALE=${4:-0.5}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for l2 in $L2S; do
    for lds in $LDSS; do
        BSMR_L2_RANGE_KB=$l2 timeout -k 10 300 python3 tools/prof_sddmm.py --iters 30 --workload reddit_like \
            --scale "$SCALE" --K 128 --lds-kb "$lds" > "$OUT/c4_${l2}_${lds}.json" 2> "$OUT/c4_${l2}_${lds}.err" || exit $?
        python3 -c "
import json; d=json.loads(open('$OUT/c4_${l2}_${lds}.json').read().strip().splitlines()[-1])
print('l2', $l2, 'lds', $lds, round(d['timing_ms']['total_ms'], 4), d['rb'])" | tee -a "$OUT/summary.txt"
    done
done
