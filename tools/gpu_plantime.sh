#!/bin/bash
# Plan-build timing (clustering) on reddit-like x0.25 / x0.5 after the plan GPU tests. Through gpurun:
#   bash tools/gpu_plantime.sh <tag>
set -o pipefail
O=gpurun_out/${1:-plantime}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu -k "plan or golden or exact or cluster" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python3 tools/plan_time.py --workload reddit_like --scale 0.25 --batches 16384 > $O/plan_c4q.json 2> $O/err.log &&
timeout -k 10 400 python3 tools/plan_time.py --workload reddit_like --scale 0.5 --batches 16384 > $O/plan_c4h.json 2>> $O/err.log
