#!/bin/bash
# The five rebuilt SuiteSparse matrices through the drop-in binary's test mode (MI355X vs the
# reference's published RTX 4090 numbers), then a rocprofv3 kernel summary of each matrix's best
# K = 128 setting. Usage through gpurun: bash tools/gpu_suitesparse.sh <tag>
set -o pipefail
TAG=${1:-ss}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1500 python3 -u tools/suitesparse_compare.py --out "$OUT" --keep-mtx > "$OUT/compare.log" 2>&1 || exit $?
for m in Trefethen_20000 Trefethen_20000b mycielskian14 mycielskian15 mycielskian16; do
    ad=$(python3 -c "import json; r=json.load(open('$OUT/compare.json'))['matrices']['$m']['K']['128']; print(r['alpha'], r['delta'])") || exit 1
    set -- $ad
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$m" -o run -- \
        ./sddmm-gpu_amd/bin/BSMR-sddmm -f "$OUT/$m.mtx" -k 128 -a "$1" -d "$2" > "$OUT/prof_$m.log" 2>&1 || exit $?
    rm -f "$OUT/$m.mtx"
done
echo done > "$OUT/rc.txt"
