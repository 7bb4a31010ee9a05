#!/bin/bash
# Round-3 eighth pass: parity + shard tests, item-scheduling A/B (cap chosen by the slot model,
# C5 epilogue prefetch) and default-layout item timelines
set -o pipefail
TAG=${1:-r03h}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*" >> "$OUT/steps.log"; }
it() {  # name, args
    local name=$1; shift
    timeout -k 10 150 python3 tools/item_trace.py --out "$OUT/it/$name" "$@" > "$OUT/it/$name.json" 2> "$OUT/it/$name.err" || return $?
    echo "$name $(tail -n 1 $OUT/it/$name.json)" >> "$OUT/it/summary.txt"
}
mkdir -p "$OUT/it"
step tests && timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shards.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 &&
step ab_sched && timeout -k 10 900 bash tools/ab_sched.sh "$TAG/ab_sched" "C2 C3 C4 C5u C5b M14 M15 M15k512 M16 M16k512 T64 T128" &&
step itemtrace && it myc15_K256 --workload mycielskian15 --K 256 --alpha 0.5 --delta 0.7 &&
it myc15_K512 --workload mycielskian15 --K 512 --alpha 0.5 --delta 0.7 &&
it myc16_K256 --workload mycielskian16 --K 256 --alpha 0.5 --delta 0.7 &&
it myc16_K512 --workload mycielskian16 --K 512 --alpha 0.5 --delta 0.7 &&
it myc14_K128 --workload mycielskian14 --K 128 --alpha 0.3 --delta 0.3 &&
it C4q --workload reddit_like --scale 0.25 --K 128 &&
step cltrace && timeout -k 10 300 python3 tools/cluster_trace.py --workload reddit_like --scale 0.25 --dump "$OUT/cl_q.npy" > "$OUT/cltrace_q.json" 2> "$OUT/cltrace_q.err" &&
timeout -k 10 300 python3 tools/cluster_trace.py --workload reddit_like --scale 1.0 --dump "$OUT/cl_x1.npy" > "$OUT/cltrace_x1.json" 2> "$OUT/cltrace_x1.err"
rc=$?
step "done rc=$rc"
echo "rc=$rc" > "$OUT/rc.txt"
exit $rc
