set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ptile.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
TR="python3 tools/trace_sddmm.py"
for t in 4 2; do
BSMR_PTILE_TPI=$t timeout -k 10 300 $TR --workload dlmc_like --mask block --K 512 --dtype bf16 --waves-per-wg 1 --dump $O/trace_ptile_tpi$t.npy > $O/trace_ptile_tpi$t.json 2> $O/trace_ptile_tpi$t.err || exit 2
done
BSMR_PTILE=0 timeout -k 10 300 $TR --workload dlmc_like --mask block --K 512 --dtype bf16 --waves-per-wg 8 --dump $O/trace_dense.npy > $O/trace_dense.json 2> $O/trace_dense.err || exit 3
timeout -k 10 300 $TR --workload nips_like --K 128 --dump $O/trace_C2_warm.npy > $O/trace_C2_warm.json 2> $O/trace_C2_warm.err || exit 4
timeout -k 10 300 $TR --workload nips_like --K 128 --cold --dump $O/trace_C2_cold.npy > $O/trace_C2_cold.json 2> $O/trace_C2_cold.err || exit 5
Q="--no-cpu-baseline --no-vendor --pmc off"
for tm in 128 96 64 0; do
  BSMR_TILE_MIN_HALF=$tm timeout -k 10 300 python3 bench.py $Q --config C3 --steps 50 --warmup 5 --no-split > $O/c3_tmh$tm.json 2> $O/c3_tmh$tm.err || exit 6
done
timeout -k 10 400 python3 tools/c4_floor.py --scale 1.0 --iters 10 > $O/c4_floor.json 2> $O/c4_floor.err || exit 7
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r06d/*.json")):
    d=json.load(open(f))
    if "value" in d: print(f.split('/')[-1], d.get("value"), d.get("ms_per_step"))
    else: print(f.split('/')[-1], json.dumps(d)[:1500])
PY
