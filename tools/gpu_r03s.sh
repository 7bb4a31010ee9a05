#!/bin/bash
# C2 per-item timelines (40 launches) for the item cost model: is the item-time spread structural?
set -o pipefail
OUT=gpurun_out/r03s
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/item_trace.py --workload nips_like --K 128 --iters 40 --out "$OUT/C2" > "$OUT/C2.json" 2> "$OUT/C2.err" &&
timeout -k 10 200 python3 tools/item_trace.py --workload mycielskian14 --K 128 --iters 20 --out "$OUT/myc14" > "$OUT/myc14.json" 2> "$OUT/myc14.err"
