#!/bin/bash
# End-of-round-3 evidence, part 2: rocprofv3 kernel summary of the C2 bench with every traced
# launch a timed step (--no-split, no cold steps), the SuiteSparse comparison (same-box CPU leg,
# roofline per point), the C4 x1 shard rehearsal and the clustering timeline.
set -o pipefail
TAG=${1:-r03r}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*" >> "$OUT/steps.log"; }
step rocprof && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_C2" -o run -- \
    python3 bench.py --no-cpu-baseline --no-vendor --pmc off --no-split --cold-steps 0 > "$OUT/bench_C2_rocprof.json" 2> "$OUT/bench_C2_rocprof.err" &&
step suitesparse && timeout -k 10 900 python3 -u tools/suitesparse_compare.py --out "$OUT/ss" > "$OUT/ss.log" 2>&1 &&
step shards && timeout -k 10 600 python3 tools/shard_sim.py --workload reddit_like --scale 1.0 --worlds 2,4,8 --rebalance 3 --local > "$OUT/shards_c4x1.json" 2> "$OUT/shards_c4x1.err" &&
step cltrace && timeout -k 10 700 bash tools/gpu_cltrace.sh "$TAG/cltrace"
rc=$?
step "done rc=$rc"
exit $rc
