#!/bin/bash
# Parameter sweep of the row-block SDDMM (through gpurun): for each "name|prof_sddmm args" line of
# the sweep file, one prof_sddmm run (dense-only / residual-only / fused timings). Usage:
#   bash tools/gpu_sweep.sh <tag> <sweep file>
set -o pipefail
TAG=${1:-sweep}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
rc=0
while IFS='|' read -r name args; do
    [ -z "$name" ] && continue
    echo "[$(date +%T)] $name: $args" >> "$OUT/steps.log"
    timeout -k 10 240 python3 tools/prof_sddmm.py --iters 50 $args > "$OUT/$name.json" 2> "$OUT/$name.err" || { rc=$?; break; }
done < "$2"
echo "rc=$rc" > "$OUT/rc.txt"
exit $rc
