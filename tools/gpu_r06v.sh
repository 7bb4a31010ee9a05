set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06v; mkdir -p $O
V="--variant rows:col_blocks=0 --variant cols: --variant split:col_blocks=1,diag=4096"
timeout -k 10 200 python3 tools/layout_ab.py --config C2 --rounds 6 $V --prespin-ms 100 --prespin-kind sleep > $O/ab_sleep.json 2> $O/ab_sleep.err || exit 1
timeout -k 10 200 python3 tools/layout_ab.py --config C2 --rounds 6 $V --prespin-ms 100 --prespin-kind mm > $O/ab_mm.json 2> $O/ab_mm.err || exit 2
timeout -k 10 200 python3 tools/layout_ab.py --config C2 --rounds 30 $V > $O/ab_long.json 2> $O/ab_long.err || exit 3
for f in $O/ab_*.json; do python3 -c "
import json; d=json.load(open('$f')); print('$f', json.dumps(d['median_us'])); print(json.dumps(d['us']))"; done
