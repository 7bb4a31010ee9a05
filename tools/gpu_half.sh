#!/bin/bash
# fp16/bf16 row-block check: parity tests, C3 (cop20k-like fp16 K=256) and C5 bench lines.
set -o pipefail
TAG=${1:-half}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q -k "half or checkdata or blocky or batch or cli" > "$OUT/pytest.log" 2>&1 || { echo "pytest rc=$?" > "$OUT/rc.txt"; exit 1; }
timeout -k 10 300 python3 bench.py --config C3 --steps 50 --warmup 5 > "$OUT/bench_C3.json" 2> "$OUT/bench_C3.err" || { echo "C3 rc=$?" > "$OUT/rc.txt"; exit 1; }
timeout -k 10 300 python3 bench.py --config C5 --steps 50 --warmup 5 > "$OUT/bench_C5u.json" 2> "$OUT/bench_C5u.err" || { echo "C5 rc=$?" > "$OUT/rc.txt"; exit 1; }
timeout -k 10 300 python3 bench.py --config C2 --steps 100 --warmup 10 --no-cpu-baseline > "$OUT/bench_C2.json" 2> "$OUT/bench_C2.err" || { echo "C2 rc=$?" > "$OUT/rc.txt"; exit 1; }
echo "rc=0" > "$OUT/rc.txt"
