#!/bin/bash
# Round evidence pass (through gpurun): smoke, GPU suite, the driver's bench line (PMC traffic in-run),
# a rocprofv3 kernel-trace of the timed bench steps, and the other BASELINE configs' bench lines.
# Every GPU step has its own time limit; the first failure ends the pass.
set -o pipefail
TAG=${1:-round}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*" >> "$OUT/steps.log"; }
step smoke && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
step pytest && timeout -k 10 900 python3 -m pytest tests -x -q -m gpu > "$OUT/pytest_gpu.log" 2>&1 &&
step bench && timeout -k 10 300 python3 bench.py > "$OUT/bench_C2.json" 2> "$OUT/bench_C2.err" &&
step rocprof && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o prof -- \
    python3 bench.py --no-cpu-baseline --no-vendor --no-split --pmc off > "$OUT/bench_C2_rocprof.json" 2> "$OUT/bench_C2_rocprof.err" &&
step C3 && timeout -k 10 600 python3 bench.py --config C3 --steps 50 --warmup 5 > "$OUT/bench_C3.json" 2> "$OUT/bench_C3.err" &&
step C5u && timeout -k 10 300 python3 bench.py --config C5 --mask uniform --steps 100 --warmup 10 > "$OUT/bench_C5u.json" 2> "$OUT/bench_C5u.err" &&
step C5b && timeout -k 10 300 python3 bench.py --config C5 --mask block --steps 100 --warmup 10 > "$OUT/bench_C5b.json" 2> "$OUT/bench_C5b.err" &&
step C4 && timeout -k 10 900 python3 bench.py --config C4 --scale 0.5 --steps 20 --warmup 3 > "$OUT/bench_C4.json" 2> "$OUT/bench_C4.err"
rc=$?
step "done rc=$rc"
echo "rc=$rc" > "$OUT/rc.txt"
exit $rc
