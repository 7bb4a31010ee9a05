#!/bin/bash
# row-block image budget sweep (bsmr_plan_options.lds_budget_kb) on nips-like per K (through gpurun)
#   bash tools/rb_size_sweep.sh <tag> "<K>:<kb> <K>:<kb> ..." [dtype]
set -o pipefail
TAG=${1:-rbsize}; PAIRS=$2; DT=${3:-f32}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for p in $PAIRS; do
    k=${p%%:*}; kb=${p##*:}
    timeout -k 10 200 python3 tools/prof_sddmm.py --iters 50 --workload nips_like --K $k --dtype $DT \
        --lds-kb $kb > "$OUT/K${k}_$kb.json" 2> "$OUT/K${k}_$kb.err" || exit $?
    echo "K=$k lds_kb=$kb $(python3 -c "import json; d=json.loads(open('$OUT/K${k}_$kb.json').read().strip().splitlines()[-1]); print(d['timing_ms']['total_ms'])")" | tee -a "$OUT/summary.txt"
done
