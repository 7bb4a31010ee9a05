#!/bin/bash
# A/B of two builds of libbsmr_amd.so on arbitrary prof_sddmm argument sets (through gpurun):
#   bash tools/ab_lib_args.sh <tag> <variant.so> "<args 1>" "<args 2>" ...
set -o pipefail
TAG=$1; VAR=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
i=0
for ARGS in "$@"; do
    i=$((i + 1))
    for v in base var base var; do
        if [ $v = var ]; then export BSMR_LIB_PATH=$VAR; else unset BSMR_LIB_PATH; fi
        timeout -k 10 300 python3 tools/prof_sddmm.py --iters 30 $ARGS > "$OUT/${i}_$v.json" 2> "$OUT/${i}_$v.err" || exit $?
        echo "[$ARGS] $v $(python3 -c "import json; d=json.loads(open('$OUT/${i}_$v.json').read().strip().splitlines()[-1]); print(d['timing_ms']['total_ms'])")" | tee -a "$OUT/summary.txt"
    done
done
