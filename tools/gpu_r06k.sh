set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06k; mkdir -p $O
Q="--no-cpu-baseline --no-vendor --pmc off"
for c in "C2" "C5 --mask uniform" "C3 --steps 50 --warmup 5"; do
  n=${c%% *}
  timeout -k 10 300 python3 bench.py $Q --config $c > $O/cold_$n.json 2> $O/cold_$n.err || exit 1
done
TR="python3 tools/trace_sddmm.py"
for m in write read; do for r in 1 2; do
timeout -k 10 300 $TR --workload nips_like --K 128 --cold $m --dump $O/trace_C2_cold_${m}_$r.npy > $O/trace_C2_cold_${m}_$r.json 2> $O/trace_C2_cold_${m}_$r.err || exit 2
done; done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r06k/cold_*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split('/')[-1], d["value"], d["ms_per_step"], json.dumps(d.get("cold")))
for f in sorted(glob.glob("gpurun_out/r06k/trace_*.json")):
    d=json.load(open(f)); print(f.split('/')[-1], {k: d.get(k) for k in ("span_us","start_us","life_us","mid_us","end_us")})
PY
