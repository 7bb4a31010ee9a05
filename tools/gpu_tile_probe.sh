#!/bin/bash
# C2 fp32 MFMA tile probe (one gpurun pass): dense / residual / fused launch times under several
# BSMR_TILE_MIN_F32 settings (ab_grid.sh), then wave timelines of the default and the all-tiles
# layouts (trace_sddmm.py: staging, first tile, piece phase per wave).
#   bash tools/gpu_tile_probe.sh <tag> [settings...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
SETS=${*:-"- TILE_MIN_F32=0 TILE_MIN_F32=128 TILE_MIN_F32=192"}
bash tools/ab_grid.sh "$TAG" C2 $SETS || exit $?
timeout -k 10 300 python3 tools/trace_sddmm.py --workload nips_like --K 128 > "$OUT/trace_default.json" 2> "$OUT/trace_default.err" || exit $?
BSMR_TILE_MIN_F32=0 timeout -k 10 300 python3 tools/trace_sddmm.py --workload nips_like --K 128 > "$OUT/trace_tiles.json" 2> "$OUT/trace_tiles.err" || exit $?
for t in 257 0 128 192; do
    BSMR_TILE_MIN_F32=$t timeout -k 10 120 python3 tools/tile_items.py > "$OUT/items_$t.json" 2>> "$OUT/items.err" || exit $?
done
