#!/bin/bash
# Round-3: new item-scheduling tests + layout variants, then the clustering timeline with the
# per-wave split (tools/cluster_trace.py)
set -o pipefail
TAG=${1:-r03j}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*" >> "$OUT/steps.log"; }
step tests && timeout -k 10 900 python3 -u -m pytest tests/test_gpu_item_sched.py "tests/test_gpu_parity.py::test_rowblock_layout_variants" -x -v --timeout 600 --timeout-method thread > "$OUT/pytest.log" 2>&1 &&
step cltrace && timeout -k 10 600 bash tools/gpu_cltrace.sh "$TAG/cltrace"
rc=$?
step "done rc=$rc"
echo "rc=$rc" > "$OUT/rc.txt"
exit $rc
