set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06p; mkdir -p $O
timeout -k 10 400 python3 tools/transpose_ab.py --reps 3 --rb-rows 256 304 --s-rb-rows 256 304 320 > $O/transpose_ab.json 2> $O/transpose_ab.err || exit 2
python3 -c "
import json; d=json.load(open('$O/transpose_ab.json')); print(json.dumps(d['median_us'])); [print(k, v['rb_rows'][2], v['rb_items'][2], v['rb_pieces'][2]) for k,v in d.items() if k.startswith('layout')]"
