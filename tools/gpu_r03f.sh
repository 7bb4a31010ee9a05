#!/bin/bash
# Round-3 sixth pass: row-block parity + shard tests, item-scheduling A/B (cap 2, capacity-split
# cost cuts), per-item timelines, C5 dense-launch wave timeline
set -o pipefail
TAG=${1:-r03f}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*" >> "$OUT/steps.log"; }
step tests && timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shards.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 &&
step ab_sched && timeout -k 10 900 bash tools/ab_sched.sh "$TAG/ab_sched" &&
step trace_c5 && timeout -k 10 120 python3 tools/trace_sddmm.py --workload dlmc_like --mask uniform --K 512 --dtype bf16 --waves-per-wg 1 > "$OUT/trace_C5u.json" 2> "$OUT/trace_C5u.err" &&
step itemcal && timeout -k 10 900 bash tools/gpu_itemcal.sh "$TAG/itemcal"
rc=$?
step "done rc=$rc"
echo "rc=$rc" > "$OUT/rc.txt"
exit $rc
