#!/bin/bash
# mycielskian K = 512 row-block sweep (rows per block x staged output), K = 256 defaults beside.
set -o pipefail
OUT=gpurun_out/r03t
mkdir -p "$OUT"
export TMPDIR=/tmp
S512='--set "" --set BSMR_RB_ROWS=32 --set BSMR_RB_ROWS=48 --set BSMR_RB_ROWS=64 --set BSMR_RB_ROWS=80 --set BSMR_RB_ROWS=32,BSMR_OUT_STAGED=0 --set BSMR_RB_ROWS=48,BSMR_OUT_STAGED=0 --set BSMR_RB_ROWS=64,BSMR_OUT_STAGED=0 --set BSMR_OUT_STAGED=1 --set BSMR_OUT_STAGED=0'
run() { eval timeout -k 10 300 python3 tools/rb_sweep.py "$@" >> "$OUT/sweep.jsonl" 2>> "$OUT/sweep.err"; }
BSMR_DIAG=1024 timeout -k 10 120 python3 tools/rb_sweep.py --workload mycielskian14 --K 128 --alpha 0.5 --delta 0.3 --set "" > "$OUT/myc14_k128_layout.txt" 2>&1 &&
run --workload mycielskian14 --K 512 --alpha 0.5 --delta 0.7 $S512 &&
run --workload mycielskian15 --K 512 --alpha 0.5 --delta 0.3 $S512 &&
run --workload mycielskian16 --K 512 --alpha 0.5 --delta 0.7 $S512 &&
run --workload mycielskian14 --K 256 --alpha 0.5 --delta 0.3 --set '""' &&
run --workload mycielskian15 --K 256 --alpha 0.3 --delta 0.1 --set '""' &&
run --workload mycielskian16 --K 256 --alpha 0.5 --delta 1.1 --set '""'
