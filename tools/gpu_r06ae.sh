set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ae; mkdir -p $O
for c in "C2" "C3 --steps 50" "C4 --scale 0.5 --steps 20"; do
  n=$(echo $c | tr -d ' .-' )
  timeout -k 10 600 python3 tools/layout_ab.py --config $c --rounds 12 --variant base: --variant earlyB:late_b=0 > $O/ab_$n.json 2> $O/ab_$n.err || { tail -5 $O/ab_$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/ab_$n.json')); print('$n', json.dumps(d['median_us'])); print(json.dumps(d['us']))"
done
