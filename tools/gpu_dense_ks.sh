#!/bin/bash
# Dense-sampled launch: one (KS=1) or two (KS=2, split-k) wave sets per tile (BSMR_DENSE_KS):
# dense GPU tests under both, C5 uniform and the 4096^2 sweep under both.
# Usage (through gpurun): bash tools/gpu_dense_ks.sh <tag>
set -o pipefail
O=gpurun_out/${1:-ks}
mkdir -p $O
export TMPDIR=/tmp
for v in 1 2; do
  BSMR_DENSE_KS=$v timeout -k 10 300 python3 -u -m pytest tests -x -q -m gpu -k "dense" --timeout 120 --timeout-method thread > $O/pytest_ks$v.log 2>&1 || exit 1
done
for r in 1 2; do for v in 1 2; do
  BSMR_DENSE_KS=$v timeout -k 10 300 python3 bench.py --config C5 --steps 100 --warmup 10 --no-cpu-baseline --no-vendor --cold-steps 0 --no-split > $O/C5u_ks${v}_$r.json 2>> $O/err.log || exit 1
done; done
for v in 1 2; do
  BSMR_DENSE_KS=$v timeout -k 10 300 python3 tools/dense_sweep.py --n 4096 --K 256 --dtype f16 --densities 0.005,0.08 > $O/sweep4096_ks$v.json 2>> $O/err.log || exit 1
  BSMR_DENSE_KS=$v timeout -k 10 300 python3 tools/dense_sweep.py --densities 0.005,0.05,0.1 > $O/sweep2048_ks$v.json 2>> $O/err.log || exit 1
done
