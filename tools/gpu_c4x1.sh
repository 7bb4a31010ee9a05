#!/bin/bash
# C4 at full size (reddit-like x1, 232 M entries, fp32 K=128) on ONE GPU: bench line with in-run PMC traffic, then a rocprofv3 kernel trace of the same bench (through gpurun).
set -o pipefail
OUT=gpurun_out/r02c4x1
mkdir -p $OUT
export TMPDIR=/tmp
echo "[$(date +%T)] bench" >> $OUT/steps.log
timeout -k 10 600 python3 bench.py --config C4 --scale 1 --steps 10 --warmup 2 --no-vendor > $OUT/bench_C4x1.json 2> $OUT/bench_C4x1.err &&
echo "[$(date +%T)] rocprof" >> $OUT/steps.log &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o prof -- python3 bench.py --config C4 --scale 1 --steps 10 --warmup 2 --no-vendor --no-cpu-baseline --no-split --pmc off > $OUT/bench_C4x1_rocprof.json 2> $OUT/bench_C4x1_rocprof.err
rc=$?
echo "[$(date +%T)] done rc=$rc" >> $OUT/steps.log
exit $rc
