#!/bin/bash
# Round-3 second pass: test-mode log fixtures from the Release CLI, C2 rocprof kernel summary,
# C3 / C5 bench lines, C4 x1 bench lines (default and two layout variants), then the C4 x1
# L2-miss attribution (tools/gpu_c4attr.sh). Every GPU step has its own limit.
set -o pipefail
TAG=${1:-r03b}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*" >> "$OUT/steps.log"; }
step plan_parity && timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q -k "plan or reference_logs or cluster" --timeout 300 --timeout-method thread > "$OUT/plan_parity.log" 2>&1 &&
step plan_ab && timeout -k 10 300 python3 tools/plan_time.py --workload reddit_like --scale 1.0 --batches 16384 > "$OUT/plan_new.json" 2> "$OUT/plan_new.err" &&
BSMR_LIB_PATH=$GRAFT_REPO_ROOT/sddmm-gpu_amd/lib_base/libbsmr_amd.so timeout -k 10 300 python3 tools/plan_time.py --workload reddit_like --scale 1.0 --batches 16384 > "$OUT/plan_base.json" 2> "$OUT/plan_base.err" &&
step testmode && timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0, 'sddmm-gpu_amd')
from bsmr import synth
M, N, rp, ci = synth.SUITESPARSE_REBUILDS['Trefethen_20000']()
import os; os.makedirs('/tmp/suiteSparse_dataset/Trefethen_20000', exist_ok=True)
synth.write_mtx('/tmp/suiteSparse_dataset/Trefethen_20000/Trefethen_20000.mtx', M, N, rp, ci)" &&
mkdir -p "$OUT/testmode_Trefethen_20000" &&
(cd /tmp && timeout -k 10 300 $GRAFT_REPO_ROOT/sddmm-gpu_amd/bin/BSMR-sddmm -f ./suiteSparse_dataset/Trefethen_20000/Trefethen_20000.mtx -t 1 -l "$GRAFT_REPO_ROOT/$OUT/testmode_Trefethen_20000/" > "$GRAFT_REPO_ROOT/$OUT/testmode.log" 2>&1) &&
step rocprof && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_C2" -o run -- \
    python3 bench.py --no-cpu-baseline --no-vendor --no-split --pmc off > "$OUT/bench_C2_rocprof.json" 2> "$OUT/bench_C2_rocprof.err" &&
step C3 && timeout -k 10 600 python3 bench.py --config C3 --steps 50 --warmup 5 --no-vendor > "$OUT/bench_C3.json" 2> "$OUT/bench_C3.err" &&
step C5u && timeout -k 10 300 python3 bench.py --config C5 --mask uniform --steps 100 --warmup 10 --no-vendor > "$OUT/bench_C5u.json" 2> "$OUT/bench_C5u.err" &&
step C5b && timeout -k 10 300 python3 bench.py --config C5 --mask block --steps 100 --warmup 10 --no-vendor > "$OUT/bench_C5b.json" 2> "$OUT/bench_C5b.err" &&
step C4 && timeout -k 10 600 python3 bench.py --config C4 --scale 1.0 --steps 20 --warmup 3 --no-vendor --cold-steps 0 > "$OUT/bench_C4x1.json" 2> "$OUT/bench_C4x1.err" &&
step C4_l2_2048 && BSMR_L2_RANGE_KB=2048 timeout -k 10 600 python3 bench.py --config C4 --scale 1.0 --steps 20 --warmup 3 --no-vendor --no-cpu-baseline --cold-steps 0 --pmc off > "$OUT/bench_C4x1_l2_2048.json" 2> "$OUT/bench_C4x1_l2_2048.err" &&
step C4_nostaged && BSMR_OUT_STAGED=0 timeout -k 10 600 python3 bench.py --config C4 --scale 1.0 --steps 20 --warmup 3 --no-vendor --no-cpu-baseline --cold-steps 0 --pmc off > "$OUT/bench_C4x1_nostaged.json" 2> "$OUT/bench_C4x1_nostaged.err" &&
step attr && bash tools/gpu_c4attr.sh "$TAG/c4attr" 1.0
rc=$?
step "done rc=$rc"
echo "rc=$rc" > "$OUT/rc.txt"
exit $rc
