set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06x; mkdir -p $O
timeout -k 10 300 python3 tools/layout_ab.py --config C2 --rounds 24 --variant rows:col_blocks=0 --variant cols304: --variant cols320:batches=0 > $O/ab.json 2> $O/ab.err || exit 1
python3 -c "
import json; d=json.load(open('$O/ab.json')); print(json.dumps(d['median_us'])); print(json.dumps(d['us'])); print(json.dumps(d['layouts']))"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_colblocks.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_cb.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_cb.log; exit 2; }
tail -1 $O/pytest_cb.log
