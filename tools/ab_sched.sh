#!/bin/bash
# A/B of the item scheduling (previous layout: BSMR_ITEM_SCHED=0 BSMR_ITEM_CAP=0) against the
# defaults on the bench configs and the SuiteSparse rebuilds: bash tools/ab_sched.sh <tag> [configs]
set -o pipefail
TAG=$1; CFGS=${2:-"C2 C3 C4 M14 M15 M15k512 M16 M16k512 T64 T128"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for c in $CFGS; do
    for v in old new old new; do
        if [ $v = old ]; then e="BSMR_ITEM_SCHED=0 BSMR_ITEM_CAP=0"; else e="BSMR_DIAG=0"; fi
        env $e timeout -k 10 300 bash tools/ab_env.sh "$TAG/raw" BSMR_DIAG 0 "$c" > /dev/null || exit $?
        echo "$c $v $(tail -n 1 $OUT/raw/summary.txt | cut -d' ' -f3-)" >> "$OUT/summary.txt"
    done
done
