#!/bin/bash
set -o pipefail
TAG=${1:-tr2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q -k "checkdata or blocky or shards or smoke" > "$OUT/pytest.log" 2>&1 || { echo "pytest rc=$?" > "$OUT/rc.txt"; exit 1; }
timeout -k 10 120 python3 tools/trace_sddmm.py --K 128 --dump "$OUT/tl_128.npy" >> "$OUT/trace.jsonl" 2>> "$OUT/err.log" || { echo "rc=1" > "$OUT/rc.txt"; exit 1; }
for K in 64 128 256 512; do
  for L in auto colmajor; do
    timeout -k 10 120 python3 tools/prof_sddmm.py --iters 50 --K $K --layout $L >> "$OUT/prof.jsonl" 2>> "$OUT/err.log" || { echo "rc=1" > "$OUT/rc.txt"; exit 1; }
  done
done
echo "rc=0" > "$OUT/rc.txt"
