#!/bin/bash
# A/B timing of two builds of libbsmr_amd.so (through gpurun): the in-tree lib vs $2 (a variant
# build, e.g. sddmm-gpu_amd/lib_exp/libbsmr_amd.so), alternating, on the listed configs.
#   bash tools/ab_lib.sh <tag> <variant.so> "C4 C3 C2" [swap]   (swap: the variant runs first)
set -o pipefail
TAG=$1; VAR=$2; CFGS=${3:-"C4 C3 C2"}; ORDER="base var base var"
[ "$4" = swap ] && ORDER="var base var base"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for c in $CFGS; do
    case "$c" in
        C2) ARGS="--workload nips_like --K 128 --dtype f32" ;;
        C3) ARGS="--workload cop20k_like --K 256 --dtype f16" ;;
        C4) ARGS="--workload reddit_like --scale 0.5 --K 128 --dtype f32" ;;
        C4x1) ARGS="--workload reddit_like --scale 1.0 --K 128 --dtype f32" ;;
        C5u) ARGS="--workload dlmc_like --mask uniform --K 512 --dtype bf16" ;;
        C5b) ARGS="--workload dlmc_like --mask block --K 512 --dtype bf16" ;;
        C2k32) ARGS="--workload nips_like --K 32 --dtype f32" ;;
        C2k512) ARGS="--workload nips_like --K 512 --dtype f32" ;;
        M15k32) ARGS="--workload mycielskian15 --K 32 --alpha 0.9 --delta 0.1" ;;
        M15k64) ARGS="--workload mycielskian15 --K 64 --alpha 0.3 --delta 0.1" ;;
        M14k256) ARGS="--workload mycielskian14 --K 256 --alpha 0.7 --delta 0.7" ;;
        M16k32) ARGS="--workload mycielskian16 --K 32 --alpha 0.3 --delta 0.1" ;;
    esac
    for v in $ORDER; do
        if [ $v = var ]; then export BSMR_LIB_PATH=$VAR; else unset BSMR_LIB_PATH; fi
        timeout -k 10 300 python3 tools/prof_sddmm.py --iters 30 $ARGS > "$OUT/${c}_$v.json" 2> "$OUT/${c}_$v.err" || exit $?
        echo "$c $v $(python3 -c "import json; d=json.loads(open('$OUT/${c}_$v.json').read().strip().splitlines()[-1]); print(d['timing_ms']['total_ms'])")" | tee -a "$OUT/summary.txt"
    done
done
