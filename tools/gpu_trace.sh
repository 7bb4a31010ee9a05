#!/bin/bash
# Wave timelines (BSMR_DIAG=32) of the SDDMM launch per layout, plus a kernel-trace of the
# profiling driver. Usage through gpurun: bash tools/gpu_trace.sh <tag>
set -o pipefail
TAG=${1:-trace}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in "colmajor 128" "auto 128" "colmajor 512" "auto 512"; do
    set -- $cfg
    timeout -k 10 120 python3 tools/trace_sddmm.py --layout $1 --K $2 --dump "$OUT/tl_$1_$2.npy" >> "$OUT/trace.jsonl" 2>> "$OUT/err.log" || { echo "trace rc=$?" > "$OUT/rc.txt"; exit 1; }
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- \
    python3 tools/prof_sddmm.py --iters 20 --K 128 > "$OUT/kt.log" 2>&1
rc=$?
echo "rc=$rc" > "$OUT/rc.txt"
exit $rc
