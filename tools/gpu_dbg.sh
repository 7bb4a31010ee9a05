#!/bin/bash
# shard launches against the host SDDMM, item scheduling on and off
set -o pipefail
OUT=gpurun_out/${1:-dbg}
mkdir -p "$OUT"
for v in 1 0; do
    BSMR_ITEM_SCHED=$v BSMR_ITEM_CAP=$v timeout -k 10 200 python3 tools/debug_shards.py > "$OUT/sched$v.json" 2> "$OUT/sched$v.err" || exit $?
done
BSMR_ITEM_SCHED=1 BSMR_ITEM_CAP=0 timeout -k 10 200 python3 tools/debug_shards.py > "$OUT/cap0.json" 2> "$OUT/cap0.err" || exit $?
BSMR_ITEM_SCHED=0 BSMR_ITEM_CAP=1 timeout -k 10 200 python3 tools/debug_shards.py > "$OUT/sched0cap1.json" 2> "$OUT/sched0cap1.err"
