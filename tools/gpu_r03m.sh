#!/bin/bash
# Round-3: clustering row chunks software-pipelined (next chunk in flight) against the previous
# build (lib_clprev) and a 128-position sub-batch variant (lib_clsub128): plan exactness tests,
# plan-time A/B and the chain timeline at reddit-like x1
set -o pipefail
TAG=${1:-r03m}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*" >> "$OUT/steps.log"; }
step tests && timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 &&
step plan_ab_half && timeout -k 10 600 bash tools/gpu_plan_ab.sh "$TAG/plan_ab" 0.5 "clprev clsub128" &&
step plan_ab_x1 && timeout -k 10 600 bash tools/gpu_plan_ab.sh "$TAG/plan_ab" 1.0 "clprev clsub128" &&
step cltrace && timeout -k 10 300 python3 tools/cluster_trace.py --workload reddit_like --scale 1.0 > "$OUT/cltrace_x1.json" 2> "$OUT/cltrace_x1.err"
rc=$?
step "done rc=$rc"
echo "rc=$rc" > "$OUT/rc.txt"
exit $rc
