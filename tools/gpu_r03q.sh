#!/bin/bash
# End-of-round-3 evidence, part 1, on the final tree: smoke, the GPU suite, the C2 bench line
# (driver's default command) and its rocprofv3 kernel summary, the C1/C3/C5/C4 x1 lines.
set -o pipefail
TAG=${1:-r03q}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*" >> "$OUT/steps.log"; }
step smoke && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
step pytest && timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
step bench && timeout -k 10 300 python3 bench.py > "$OUT/bench_C2.json" 2> "$OUT/bench_C2.err" &&
step rocprof && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_C2" -o run -- \
    python3 bench.py --no-cpu-baseline --no-vendor --pmc off > "$OUT/bench_C2_rocprof.json" 2> "$OUT/bench_C2_rocprof.err" &&
step C1 && timeout -k 10 300 python3 bench.py --config C1 > "$OUT/bench_C1.json" 2> "$OUT/bench_C1.err" &&
step C3 && timeout -k 10 600 python3 bench.py --config C3 --steps 50 --warmup 5 > "$OUT/bench_C3.json" 2> "$OUT/bench_C3.err" &&
step C5u && timeout -k 10 300 python3 bench.py --config C5 --mask uniform --steps 100 --warmup 10 > "$OUT/bench_C5u.json" 2> "$OUT/bench_C5u.err" &&
step C5b && timeout -k 10 300 python3 bench.py --config C5 --mask block --steps 100 --warmup 10 > "$OUT/bench_C5b.json" 2> "$OUT/bench_C5b.err" &&
step C4 && timeout -k 10 600 python3 bench.py --config C4 --scale 1.0 --steps 20 --warmup 3 --cold-steps 0 > "$OUT/bench_C4x1.json" 2> "$OUT/bench_C4x1.err"
rc=$?
step "done rc=$rc"
exit $rc
