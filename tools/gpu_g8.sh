#!/bin/bash
set -o pipefail
TAG=${1:-g8}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q -k "half or checkdata or batch or blocky" > "$OUT/pytest.log" 2>&1 &&
for K in 64 128 256 512; do
  timeout -k 10 120 python3 tools/prof_sddmm.py --iters 50 --K $K > "$OUT/k$K.json" 2>>"$OUT/err.log" || exit 1
done &&
timeout -k 10 120 python3 tools/prof_sddmm.py --iters 50 --K 512 --workload dlmc_like --dtype bf16 > "$OUT/c5.json" 2>>"$OUT/err.log" &&
timeout -k 10 300 python3 tools/prof_sddmm.py --workload cop20k_like --dtype f16 --K 256 --iters 20 > "$OUT/c3.json" 2>> "$OUT/err.log" &&
timeout -k 10 120 python3 abtest/old/tools/prof_sddmm.py --iters 100 --K 128 > "$OUT/old_c2.json" 2>>"$OUT/err.log" &&
timeout -k 10 120 python3 tools/prof_sddmm.py --iters 100 --K 128 > "$OUT/new_c2.json" 2>>"$OUT/err.log"
echo "rc=$?" > "$OUT/rc.txt"
