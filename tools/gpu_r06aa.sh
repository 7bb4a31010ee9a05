set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06aa; mkdir -p $O
timeout -k 10 600 python3 tools/layout_ab.py --config C4 --scale 1.0 --steps 10 --rounds 5 \
  --variant pairs: --variant nopairs:diag=16384 --variant bL2:diag=64 --variant nostore:diag=128 --variant stage:diag=8 > $O/c4_ablate.json 2> $O/c4_ablate.err || { tail -5 $O/c4_ablate.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/c4_ablate.json')); print(json.dumps(d['median_us'])); print(json.dumps(d['us']))"
