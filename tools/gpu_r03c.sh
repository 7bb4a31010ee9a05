#!/bin/bash
# Round-3 third pass: A/B of nt A staging (BSMR_STAGE_NT) on C4 x1 / C4 x0.5 / C3 / C2, the C4 x1
# FETCH_SIZE with it, the 8-way global-split rehearsal with measured-cost re-cutting, the
# SuiteSparse comparison (CPU leg + roofline per point) and a C2 wave timeline.
set -o pipefail
TAG=${1:-r03c}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*" >> "$OUT/steps.log"; }
step plan_ab && timeout -k 10 600 bash tools/gpu_plan_ab.sh "$TAG/plan_ab" 0.5 "sub128 sub256" &&
step ab_nt && timeout -k 10 900 bash tools/ab_env.sh "$TAG/ab_nt" BSMR_STAGE_NT "0 1 0 1" "C4x1 C4 C3 C2" &&
step fetch_nt && BSMR_STAGE_NT=1 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_sddmm --output-format csv \
    -d "$OUT/fetch_nt" -o run -- python3 tools/prof_sddmm.py --iters 3 --workload reddit_like --scale 1.0 > "$OUT/fetch_nt.log" 2>&1 &&
step shards && timeout -k 10 600 python3 tools/shard_sim.py --workload reddit_like --scale 1.0 --worlds 2,4,8 --rebalance 3 --local > "$OUT/shards_c4x1.json" 2> "$OUT/shards_c4x1.err" &&
step trace && timeout -k 10 300 python3 tools/trace_sddmm.py --workload nips_like > "$OUT/trace_C2.json" 2> "$OUT/trace_C2.err" &&
step suitesparse && timeout -k 10 1200 python3 -u tools/suitesparse_compare.py --out "$OUT/ss" > "$OUT/ss.log" 2>&1
rc=$?
step "done rc=$rc"
echo "rc=$rc" > "$OUT/rc.txt"
exit $rc
