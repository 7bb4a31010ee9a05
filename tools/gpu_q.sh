#!/bin/bash
# quick C2 timing + timeline
set -o pipefail
TAG=${1:-q}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/trace_sddmm.py --K 128 --dump "$OUT/tl.npy" > "$OUT/trace.json" 2>> "$OUT/err.log" &&
timeout -k 10 120 python3 tools/prof_sddmm.py --iters 50 --K 128 > "$OUT/prof.json" 2>> "$OUT/err.log"
echo "rc=$?" > "$OUT/rc.txt"
