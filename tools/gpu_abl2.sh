#!/bin/bash
set -o pipefail
TAG=${1:-abl2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for d in 0 1 2 4 6 7; do
    BSMR_DIAG=$d timeout -k 10 120 python3 tools/prof_sddmm.py --iters 50 --K 128 > "$OUT/diag_$d.json" 2>> "$OUT/err.log" || { echo "rc=1" > "$OUT/rc.txt"; exit 1; }
done

echo "rc=0" > "$OUT/rc.txt"
