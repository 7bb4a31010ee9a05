mkdir -p gpurun_out/dbg2
for w in "mycielskian15 --K 256 --alpha 0.5 --delta 0.7" "Trefethen_20000 --K 64 --alpha 0.1 --delta 0.5" "nips_like --K 128"; do
  n=$(echo $w | cut -d' ' -f1)
  BSMR_DIAG=1024 timeout -k 10 120 python3 tools/item_trace.py --workload $w --iters 3 --out gpurun_out/dbg2/$n > gpurun_out/dbg2/$n.json 2> gpurun_out/dbg2/$n.err || exit $?
done
