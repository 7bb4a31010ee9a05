#!/bin/bash
# Column-range size sweep (BSMR_L2_RANGE_KB) on the reference's matrices at their best (alpha,
# delta) per K, and C2.
set -o pipefail
OUT=gpurun_out/r03u
mkdir -p "$OUT"
export TMPDIR=/tmp
S='--set "" --set BSMR_L2_RANGE_KB=1024 --set BSMR_L2_RANGE_KB=4096 --set BSMR_L2_RANGE_KB=8192'
run() { eval timeout -k 10 300 python3 tools/rb_sweep.py "$@" $S >> "$OUT/sweep.jsonl" 2>> "$OUT/sweep.err"; }
run --workload mycielskian14 --K 512 --alpha 0.5 --delta 0.7 &&
run --workload mycielskian14 --K 256 --alpha 0.5 --delta 0.3 &&
run --workload mycielskian14 --K 128 --alpha 0.5 --delta 0.3 &&
run --workload mycielskian15 --K 512 --alpha 0.5 --delta 0.3 &&
run --workload mycielskian15 --K 256 --alpha 0.3 --delta 0.1 &&
run --workload mycielskian15 --K 128 --alpha 0.9 --delta 0.1 &&
run --workload mycielskian16 --K 512 --alpha 0.5 --delta 0.7 &&
run --workload mycielskian16 --K 256 --alpha 0.5 --delta 1.1 &&
run --workload mycielskian16 --K 128 --alpha 0.3 --delta 0.1 &&
run --workload Trefethen_20000 --K 128 --alpha 0.5 --delta 1.1 &&
run --workload Trefethen_20000 --K 512 --alpha 0.7 --delta 0.1
