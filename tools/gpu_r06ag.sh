set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ag; mkdir -p $O
for c in C5u C5b; do
  timeout -k 10 300 python3 tools/layout_ab.py --config $c --rounds 12 --variant base: --variant d2:diag=16777216 > $O/ab_$c.json 2> $O/ab_$c.err || { tail -5 $O/ab_$c.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/ab_$c.json')); print('$c', json.dumps(d['median_us']), d['checkData_errors_vs_first']); print(json.dumps(d['us']))"
done
timeout -k 10 300 python3 tools/layout_ab.py --config C5u --K 256 --rounds 12 --variant base: --variant d2:diag=16777216 > $O/ab_C5u256.json 2> $O/ab_C5u256.err || exit 2
python3 -c "
import json; d=json.load(open('$O/ab_C5u256.json')); print('C5u K256', json.dumps(d['median_us']), d['checkData_errors_vs_first'])"
