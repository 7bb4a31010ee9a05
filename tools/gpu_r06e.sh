set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06e; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ptile.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
TR="python3 tools/trace_sddmm.py"
BSMR_PTILE_TPI=4 timeout -k 10 300 $TR --workload dlmc_like --mask block --K 512 --dtype bf16 --waves-per-wg 1 > $O/trace_ptile_tpi4.json 2> $O/trace_ptile_tpi4.err || exit 2
Q="--no-cpu-baseline --no-vendor --pmc off --config C5 --steps 100 --warmup 10"
run() { local name=$1; shift; env "$@" timeout -k 10 300 python3 bench.py $Q $EXTRA > $O/$name.json 2> $O/$name.err || exit 3; }
for t in 2 3 4 5; do EXTRA="--mask block" run blk_tpi$t BSMR_PTILE_TPI=$t; done
EXTRA="--mask block" run blk_off BSMR_PTILE=0
for K in 128 256; do EXTRA="--mask block --K $K" run blk_K${K} BSMR_PTILE_TPI=4; EXTRA="--mask block --K $K" run blk_K${K}_off BSMR_PTILE=0; done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r06e/*.json")):
    d=json.load(open(f))
    if "value" in d: print(f.split('/')[-1], d.get("value"), d.get("ms_per_step"))
    else: print(f.split('/')[-1], {k: d.get(k) for k in ("span_us","mid_us","dense_us","tail_us","end_us")})
PY
