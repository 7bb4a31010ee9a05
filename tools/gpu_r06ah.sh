set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ah; mkdir -p $O
for k in 128 32 512; do
  timeout -k 10 300 python3 tools/layout_ab.py --config C2 --K $k --rounds 14 --variant lite: --variant full:diag=33554432 > $O/ab_C2k$k.json 2> $O/ab_C2k$k.err || { tail -5 $O/ab_C2k$k.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/ab_C2k$k.json')); print('C2 K$k', json.dumps(d['median_us']), d['checkData_errors_vs_first']); print(json.dumps(d['us']))"
done
Q="--no-cpu-baseline --no-vendor --pmc off --config C2"
for r in 1 2; do
  timeout -k 10 200 python3 bench.py $Q >> $O/c2_lite.json 2>> $O/c2_lite.err || exit 2
  BSMR_DIAG=33554432 timeout -k 10 200 python3 bench.py $Q >> $O/c2_full.json 2>> $O/c2_full.err || exit 3
done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r06ah/c2_*.json")):
    v=[json.loads(l) for l in open(f)]
    print(f.split('/')[-1], [round(d["ms_per_step"]*1e3,2) for d in v], [d["cold"]["ms_per_step"]*1e3 for d in v], [d["cold"]["clean"]["ms_per_step"]*1e3 for d in v], v[0]["roofline"]["kernel"][:30])
PY
