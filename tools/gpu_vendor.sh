#!/bin/bash
# rocSPARSE baseline pass (through gpurun): vendor GPU test, then bench lines with the
# vendor_baseline leg for C2, C3, C5 (uniform). First failure ends the pass.
set -o pipefail
OUT=gpurun_out/${1:-vendor}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_vendor.py -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline --cold-steps 0 > "$OUT/bench_C2.json" 2> "$OUT/bench_C2.err" &&
timeout -k 10 600 python3 bench.py --config C3 --steps 50 --warmup 5 --no-cpu-baseline --cold-steps 0 > "$OUT/bench_C3.json" 2> "$OUT/bench_C3.err" &&
timeout -k 10 300 python3 bench.py --config C5 --mask uniform --steps 100 --warmup 10 --no-cpu-baseline --cold-steps 0 > "$OUT/bench_C5u.json" 2> "$OUT/bench_C5u.err"
rc=$?
echo "rc=$rc" > "$OUT/rc.txt"
exit $rc
