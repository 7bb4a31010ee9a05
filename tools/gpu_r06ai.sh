set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ai; mkdir -p $O
timeout -k 10 300 python3 tools/layout_ab.py --config C3 --steps 50 --rounds 12 --variant lite: --variant full:diag=33554432 > $O/ab_C3.json 2> $O/ab_C3.err || { tail -5 $O/ab_C3.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/ab_C3.json')); print('C3', json.dumps(d['median_us']), d['checkData_errors_vs_first'], d['layouts'])"
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu -k "rb or batches or parity or item_sched or colblocks" --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
timeout -k 10 900 python3 -u tools/perf_guard.py --check profiles/perf_baseline.json --out $O/guard.json > $O/guard.log 2>&1; rc=$?; tail -30 $O/guard.log; exit $rc
