#!/bin/bash
# Row-block layout check: parity tests of the SDDMM paths, then timings and wave timelines.
set -o pipefail
TAG=${1:-rb}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q -k "checkdata or blocky or shards or smoke" > "$OUT/pytest.log" 2>&1 || { echo "pytest rc=$?" > "$OUT/rc.txt"; exit 1; }
for cfg in "colmajor 0 128" "auto 0 128" "auto 96 128" "auto 64 128" "colmajor 0 64" "auto 0 64"; do
    set -- $cfg
    timeout -k 10 120 python3 tools/prof_sddmm.py --iters 50 --K $3 --layout $1 --lds-kb $2 >> "$OUT/prof.jsonl" 2>> "$OUT/err.log" || { echo "prof rc=$?" > "$OUT/rc.txt"; exit 1; }
done
timeout -k 10 120 python3 tools/trace_sddmm.py --layout auto --K 128 --dump "$OUT/tl_auto_128.npy" >> "$OUT/trace.jsonl" 2>> "$OUT/err.log" || { echo "trace rc=$?" > "$OUT/rc.txt"; exit 1; }
echo "rc=0" > "$OUT/rc.txt"
