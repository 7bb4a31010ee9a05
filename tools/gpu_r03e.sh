#!/bin/bash
# Round-3 fifth pass: row-block parity + shard tests on the item-scheduling change, then its A/B
# (BSMR_ITEM_CAP + BSMR_ITEM_SCHED both 0 = the previous layout) on the bench configs and the
# reference's SuiteSparse matrices, and the per-item timelines under the new layout.
set -o pipefail
TAG=${1:-r03e}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*" >> "$OUT/steps.log"; }
step tests && timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shards.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 &&
step ab_sched && timeout -k 10 900 bash tools/ab_env.sh "$TAG/ab_sched" BSMR_ITEM_CAP,BSMR_ITEM_SCHED "0 1 0 1" "C2 C3 C4 M14 M15 M15k512 M16 M16k512 T64 T128" &&
step ab_ns && timeout -k 10 600 bash tools/ab_env.sh "$TAG/ab_dense_ns" BSMR_DENSE_NS "2 3 4 2 3 4" "C5u C5b" &&
step itemcal && timeout -k 10 900 bash tools/gpu_itemcal.sh "$TAG/itemcal"
rc=$?
step "done rc=$rc"
echo "rc=$rc" > "$OUT/rc.txt"
exit $rc
