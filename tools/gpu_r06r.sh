set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06r; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_colblocks.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_cb.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_cb.log; exit 1; }
tail -2 $O/pytest_cb.log
Q="--no-cpu-baseline --no-vendor --pmc off --no-split --config C2"
for r in 1 2 3; do
  BSMR_COL_BLOCKS=0 timeout -k 10 200 python3 bench.py $Q >> $O/c2_cb0.json 2>> $O/c2_cb0.err || exit 2
  timeout -k 10 200 python3 bench.py $Q >> $O/c2_auto.json 2>> $O/c2_auto.err || exit 3
  BSMR_RB_ROWS=288 timeout -k 10 200 python3 bench.py $Q >> $O/c2_rb288.json 2>> $O/c2_rb288.err || exit 4
done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r06r/*.json")):
    v=[json.loads(l) for l in open(f)]
    print(f.split('/')[-1], [round(d["ms_per_step"]*1e3,2) for d in v], v[0]["config"]["rowblock_layout"])
PY
