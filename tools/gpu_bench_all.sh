#!/bin/bash
# Bench lines of every BASELINE config (in-run PMC traffic each) and a rocprofv3 kernel-trace of
# the driver's C2 line (through gpurun): bash tools/gpu_bench_all.sh <tag>
set -o pipefail
TAG=${1:-bench}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*" >> "$OUT/steps.log"; }
step C2 && timeout -k 10 300 python3 bench.py > "$OUT/bench_C2.json" 2> "$OUT/bench_C2.err" &&
step rocprof && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o prof -- \
    python3 bench.py --no-cpu-baseline --no-vendor --no-split --pmc off > "$OUT/bench_C2_rocprof.json" 2> "$OUT/bench_C2_rocprof.err" &&
step C3 && timeout -k 10 600 python3 bench.py --config C3 --steps 50 --warmup 5 > "$OUT/bench_C3.json" 2> "$OUT/bench_C3.err" &&
step C5u && timeout -k 10 300 python3 bench.py --config C5 --mask uniform --steps 100 --warmup 10 > "$OUT/bench_C5u.json" 2> "$OUT/bench_C5u.err" &&
step C5b && timeout -k 10 300 python3 bench.py --config C5 --mask block --steps 100 --warmup 10 > "$OUT/bench_C5b.json" 2> "$OUT/bench_C5b.err" &&
step C4 && timeout -k 10 900 python3 bench.py --config C4 --scale 0.5 --steps 20 --warmup 3 > "$OUT/bench_C4.json" 2> "$OUT/bench_C4.err"
rc=$?
step "done rc=$rc"
echo "rc=$rc" > "$OUT/rc.txt"
exit $rc
