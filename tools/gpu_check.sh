#!/bin/bash
# One GPU-box pass: smoke, GPU parity tests, bench, rocprofv3 kernel-trace summary of the bench
# (timed steps only: --no-split), PMC traffic passes. Usage (from the repo root, through gpurun):
#   bash tools/gpu_check.sh [tag] [pytest -k expr]
# Every GPU step has its own time limit and the steps are chained with &&, so the first
# failure (or fault, abort, timeout) ends the pass.
set -o pipefail
TAG=${1:-r01}
KEXPR=${2:-}
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
PYK=()
if [ -n "$KEXPR" ]; then PYK=(-k "$KEXPR"); fi

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1 &&
timeout -k 10 900 python -m pytest tests -x -q -m gpu "${PYK[@]}" > "$OUT/pytest_gpu_$TAG.log" 2>&1 &&
bash tools/gpu_pmc.sh "pmc_$TAG" 128 &&
python3 tools/pmc_traffic.py "$OUT/pmc_$TAG" profiles/traffic_C2_K128.json > "$OUT/traffic_$TAG.json" &&
timeout -k 10 300 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o prof -- \
    python3 bench.py --no-cpu-baseline --no-vendor --no-split > "$OUT/bench_prof_$TAG.json" 2> "$OUT/bench_prof_$TAG.err"
rc=$?
echo "gpu_check rc=$rc" > "$OUT/gpu_check_$TAG.rc"
exit $rc
