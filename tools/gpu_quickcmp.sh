#!/bin/bash
# Quick A/B pass after a kernel change (through gpurun): GPU parity suite, then C2 / C3 / C4 x0.5
# bench lines (no vendor leg). Every GPU step has its own time limit; the first failure ends it.
#   bash tools/gpu_quickcmp.sh <tag>
set -o pipefail
O=gpurun_out/${1:-quick}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python3 -m pytest tests -x -q -m gpu > "$O/pytest_gpu.log" 2>&1 &&
timeout -k 10 300 python3 bench.py --no-vendor > "$O/bench_C2.json" 2> "$O/bench_C2.err" &&
timeout -k 10 300 python3 bench.py --config C3 --steps 50 --warmup 5 --no-cpu-baseline --no-vendor \
    > "$O/bench_C3.json" 2> "$O/bench_C3.err" &&
timeout -k 10 300 python3 bench.py --config C5 --mask uniform --steps 100 --warmup 10 --no-cpu-baseline --no-vendor \
    > "$O/bench_C5u.json" 2> "$O/bench_C5u.err" &&
timeout -k 10 600 python3 bench.py --config C4 --scale 0.5 --steps 20 --warmup 3 --no-cpu-baseline --no-vendor \
    > "$O/bench_C4.json" 2> "$O/bench_C4.err" &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-vendor > "$O/bench_C2b.json" 2> "$O/bench_C2b.err"
rc=$?
echo "rc=$rc" > "$O/rc.txt"
exit $rc
