#!/bin/bash
# run prof_sddmm of each tree (its own binding and library) on two mycielskian settings, alternating
set -o pipefail
OUT=gpurun_out/r04zs; mkdir -p $OUT
for rep in 1 2; do
for t in exp_old/3e19a14 exp_old/d26e2eb exp_old/74c5458 .; do
  for cfg in "mycielskian15 64 0.3 0.1" "mycielskian16 128 0.3 0.1"; do
    set -- $cfg
    (cd $t && timeout -k 10 200 python3 tools/prof_sddmm.py --iters 50 --workload $1 --K $2 --alpha $3 --delta $4) > $OUT/run.json 2>> $OUT/err.log || exit $?
    echo "$t $1 K=$2 $(python3 -c "import json; d=json.loads(open('$OUT/run.json').read().strip().splitlines()[-1]); print(d['timing_ms']['total_ms'], d.get('rb',{}).get('rb_items'), d.get('rb',{}).get('rb_pieces'))")" | tee -a $OUT/summary.txt
  done
done
done
