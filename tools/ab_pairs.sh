#!/bin/bash
# pairs on / off (BSMR_DIAG & 16384) over staged-output configs: bash tools/ab_pairs.sh <tag> cfg...
set -o pipefail
TAG=$1; shift
for c in "$@"; do
    timeout -k 10 300 bash tools/ab_grid.sh "$TAG" "$c" - DIAG=16384 || exit $?
done
