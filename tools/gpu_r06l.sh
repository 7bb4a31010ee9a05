set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06l; mkdir -p $O
timeout -k 10 120 tools/ubench/launch_floor > $O/launch_floor.json 2> $O/launch_floor.err || exit 1
Q="--no-cpu-baseline --no-vendor --pmc off --no-split"
for p in 0 1 0 1; do
  BSMR_PTILE=$p timeout -k 10 300 python3 bench.py $Q --config C5 --mask uniform --steps 100 --warmup 10 >> $O/c5u_ptile$p.json 2>> $O/c5u_ptile$p.err || exit 2
done
cat $O/launch_floor.json
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r06l/c5u_*.json")):
    for l in open(f):
        d=json.loads(l); print(f.split('/')[-1], d["value"], d["ms_per_step"], d["roofline"]["kernel"][:60])
PY
