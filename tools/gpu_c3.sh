#!/bin/bash
set -o pipefail
TAG=${1:-c3}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q -k "half or checkdata or batch" > "$OUT/pytest.log" 2>&1 &&
timeout -k 10 300 python3 tools/trace_sddmm.py --workload cop20k_like --dtype f16 --K 256 > "$OUT/trace_c3.json" 2>> "$OUT/err.log" &&
timeout -k 10 300 python3 tools/prof_sddmm.py --workload cop20k_like --dtype f16 --K 256 --iters 20 > "$OUT/prof_c3.json" 2>> "$OUT/err.log" &&
timeout -k 10 120 python3 abtest/old/tools/prof_sddmm.py --iters 100 --K 128 > "$OUT/old_c2.json" 2>>"$OUT/err.log" &&
timeout -k 10 120 python3 tools/prof_sddmm.py --iters 100 --K 128 > "$OUT/new_c2.json" 2>>"$OUT/err.log"
echo "rc=$?" > "$OUT/rc.txt"
