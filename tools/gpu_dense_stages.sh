#!/bin/bash
# Dense-sampled launch variants (BSMR_DENSE_KC / BSMR_DENSE_STAGES) on the sweep shapes and C5,
# after the dense GPU tests under each. Usage (through gpurun): bash tools/gpu_dense_stages.sh <tag>
set -o pipefail
O=gpurun_out/${1:-stages}
mkdir -p $O
export TMPDIR=/tmp
for v in "64 2" "32 2" "32 3" "32 4"; do
  set -- $v
  export BSMR_DENSE_KC=$1 BSMR_DENSE_STAGES=$2
  t=kc$1_s$2
  timeout -k 10 300 python3 -u -m pytest tests -x -q -m gpu -k "dense" --timeout 120 --timeout-method thread > $O/pytest_$t.log 2>&1 &&
  timeout -k 10 300 python3 tools/dense_sweep.py --densities 0.005,0.05,0.1 > $O/sweep_2048_512_$t.json 2>> $O/err.log &&
  timeout -k 10 300 python3 tools/dense_sweep.py --n 4096 --K 256 --dtype f16 --densities 0.005,0.08 > $O/sweep_4096_256_$t.json 2>> $O/err.log &&
  timeout -k 10 300 python3 bench.py --config C5 --steps 50 --warmup 5 --no-cpu-baseline --no-vendor --cold-steps 0 > $O/C5u_$t.json 2>> $O/err.log || exit 1
done
