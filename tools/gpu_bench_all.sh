#!/bin/bash
# Bench lines of every BASELINE config (in-run PMC traffic each) and a rocprofv3 kernel-trace
# summary of each config's timed steps (through gpurun): bash tools/gpu_bench_all.sh <tag>
set -o pipefail
TAG=${1:-bench}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*" >> "$OUT/steps.log"; }
prof() {  # $1 = name, rest = bench args
    local name=$1; shift
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" -o prof -- \
        python3 bench.py --no-cpu-baseline --no-vendor --no-split --pmc off "$@" > "$OUT/rocprof_$name.json" 2> "$OUT/rocprof_$name.err"
}
step C2 && timeout -k 10 300 python3 bench.py > "$OUT/bench_C2.json" 2> "$OUT/bench_C2.err" &&
step C2prof && prof C2 &&
step C3 && timeout -k 10 600 python3 bench.py --config C3 --steps 50 --warmup 5 > "$OUT/bench_C3.json" 2> "$OUT/bench_C3.err" &&
step C3prof && prof C3 --config C3 --steps 50 --warmup 5 &&
step C5u && timeout -k 10 300 python3 bench.py --config C5 --mask uniform --steps 100 --warmup 10 > "$OUT/bench_C5u.json" 2> "$OUT/bench_C5u.err" &&
step C5uprof && prof C5u --config C5 --mask uniform --steps 100 --warmup 10 &&
step C5b && timeout -k 10 300 python3 bench.py --config C5 --mask block --steps 100 --warmup 10 > "$OUT/bench_C5b.json" 2> "$OUT/bench_C5b.err" &&
step C5bprof && prof C5b --config C5 --mask block --steps 100 --warmup 10 &&
step C4 && timeout -k 10 900 python3 bench.py --config C4 --scale 0.5 --steps 20 --warmup 3 > "$OUT/bench_C4.json" 2> "$OUT/bench_C4.err" &&
step C4prof && prof C4 --config C4 --scale 0.5 --steps 20 --warmup 3
rc=$?
step "done rc=$rc"
echo "rc=$rc" > "$OUT/rc.txt"
exit $rc
