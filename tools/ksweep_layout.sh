#!/bin/bash
# nips-like K sweep, row-block (auto) vs column-major launch (through gpurun)
#   bash tools/ksweep_layout.sh <tag> ["32 64 128 256 512"] [dtype]
set -o pipefail
TAG=${1:-ksweep}; KS=${2:-"32 64 128 256 512"}; DT=${3:-f32}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for k in $KS; do
    for lay in auto colmajor; do
        timeout -k 10 200 python3 tools/prof_sddmm.py --iters 50 --workload nips_like --K $k --dtype $DT \
            --layout $lay > "$OUT/K${k}_$lay.json" 2> "$OUT/K${k}_$lay.err" || exit $?
        echo "K=$k $lay $(python3 -c "import json; d=json.loads(open('$OUT/K${k}_$lay.json').read().strip().splitlines()[-1]); print(d['timing_ms']['total_ms'])")" | tee -a "$OUT/summary.txt"
    done
done
