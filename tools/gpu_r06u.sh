set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06u; mkdir -p $O
timeout -k 10 400 python3 tools/layout_ab.py --config C2 --rounds 9 --variant rows:col_blocks=0 --variant cols: --variant split:col_blocks=1,diag=4096 --variant orig304:col_blocks=0,orig_rows=1,rb_rows=304 > $O/layout_ab_C2.json 2> $O/layout_ab_C2.err || exit 1
python3 -c "
import json; d=json.load(open('$O/layout_ab_C2.json')); print(json.dumps(d['median_us'])); print(json.dumps(d['us'])); print(json.dumps(d['layouts']))"
