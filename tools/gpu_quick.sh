#!/bin/bash
# Quick check after a kernel/layout change (through gpurun): GPU test suite, then the bench lines
# of C2 (K = 128, 32), C3, C5 (uniform) and a reddit-like x0.25 timing. Usage: bash tools/gpu_quick.sh <tag>
set -o pipefail
O=gpurun_out/${1:-quick}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-vendor > $O/C2.json 2>> $O/err.log &&
timeout -k 10 300 python3 bench.py --K 32 --steps 100 --no-cpu-baseline --no-vendor --cold-steps 0 > $O/C2_K32.json 2>> $O/err.log &&
timeout -k 10 300 python3 bench.py --config C3 --steps 30 --warmup 5 --no-cpu-baseline --no-vendor --cold-steps 0 > $O/C3.json 2>> $O/err.log &&
timeout -k 10 300 python3 bench.py --config C5 --steps 50 --warmup 5 --no-cpu-baseline --no-vendor --cold-steps 0 > $O/C5u.json 2>> $O/err.log &&
timeout -k 10 300 python3 tools/prof_sddmm.py --iters 10 --workload reddit_like --scale 0.25 > $O/C4q.json 2>> $O/err.log
