#!/bin/bash
# Dense-sampled launch check (through gpurun): half-precision GPU tests, then the C5 bench lines
# and a density sweep of dense-sampled vs gathered launches. Usage: bash tools/gpu_dense.sh <tag>
set -o pipefail
O=gpurun_out/${1:-dense}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu -k "half or dense or dlmc or blocky" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --config C5 --steps 50 --warmup 5 --no-cpu-baseline --no-vendor --cold-steps 0 > $O/C5u.json 2>> $O/err.log &&
timeout -k 10 300 python3 bench.py --config C5 --mask block --steps 50 --warmup 5 --no-cpu-baseline --no-vendor --cold-steps 0 > $O/C5b.json 2>> $O/err.log &&
timeout -k 10 300 python3 tools/dense_sweep.py > $O/sweep_2048_512.json 2>> $O/err.log &&
timeout -k 10 300 python3 tools/dense_sweep.py --n 4096 --K 256 --dtype f16 --densities 0.005,0.01,0.02,0.04,0.08 > $O/sweep_4096_256.json 2>> $O/err.log
