#!/bin/bash
# Round-3 fourth pass: A/B of late phase-0 B loads (BSMR_LATE_B) and one item per segment
# (BSMR_SEG_ITEMS), then the K-anomaly sweep (tools/gpu_ksweep.sh).
set -o pipefail
TAG=${1:-r03d}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*" >> "$OUT/steps.log"; }
step ab_lateb && timeout -k 10 900 bash tools/ab_env.sh "$TAG/ab_lateb" BSMR_LATE_B "0 1 0 1" "C2 C3 C4 C5u" &&
step ab_seg && timeout -k 10 900 bash tools/ab_env.sh "$TAG/ab_seg" BSMR_SEG_ITEMS "0 1 0 1" "C4x1 C4" &&
step ksweep && timeout -k 10 1000 bash tools/gpu_ksweep.sh "$TAG/ksweep"
rc=$?
step "done rc=$rc"
echo "rc=$rc" > "$OUT/rc.txt"
exit $rc
