set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06a; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ptile.py tests/test_gpu_plan_check.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
Q="--no-cpu-baseline --no-vendor --pmc off --config C5"
for m in block uniform; do
  timeout -k 10 300 python3 bench.py $Q --mask $m --steps 100 --warmup 10 > $O/c5${m}_auto.json 2> $O/c5${m}_auto.err || exit 2
done
BSMR_PTILE=0 timeout -k 10 300 python3 bench.py $Q --mask block --steps 100 --warmup 10 > $O/c5block_off.json 2> $O/c5block_off.err || exit 3
for t in 4 16; do BSMR_PTILE_TPI=$t timeout -k 10 300 python3 bench.py $Q --mask block --steps 100 --warmup 10 > $O/c5block_tpi$t.json 2> $O/c5block_tpi$t.err || exit 4; done
for K in 128 256; do
  timeout -k 10 300 python3 bench.py $Q --mask block --K $K --steps 100 --warmup 10 > $O/c5block_K${K}.json 2> $O/c5block_K${K}.err || exit 5
  BSMR_PTILE=0 timeout -k 10 300 python3 bench.py $Q --mask block --K $K --steps 100 --warmup 10 > $O/c5block_K${K}_off.json 2> $O/c5block_K${K}_off.err || exit 6
done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r06a/*.json")):
    try: d=json.load(open(f))
    except Exception as e: print(f, "ERR", e); continue
    print(f.split('/')[-1], d.get("value"), d.get("ms_per_step"), d.get("mfma",{}).get("launch"), d.get("kernel"))
PY
