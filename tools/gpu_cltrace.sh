#!/bin/bash
# clustering chain timeline (tools/cluster_trace.py) on reddit-like x0.25 and x1
set -o pipefail
OUT=gpurun_out/${1:-cltrace}
mkdir -p "$OUT"
for s in 0.25 1.0; do
    timeout -k 10 300 python3 tools/cluster_trace.py --workload reddit_like --scale $s --dump "$OUT/cl_$s.npy" > "$OUT/cl_$s.json" 2> "$OUT/cl_$s.err" || exit $?
done
