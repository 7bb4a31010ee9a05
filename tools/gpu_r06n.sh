set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06n; mkdir -p $O
Q="--no-cpu-baseline --no-vendor --pmc off --no-split --config C2"
run() { # name env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py $Q >> $O/$n.json 2>> $O/$n.err || exit 1
}
for r in 1 2; do
  run base BSMR_DIAG=0
  run keep BSMR_TILE_MIN_F32=0
  run keep_b0 BSMR_TILE_MIN_F32=0 BSMR_DIAG=8388608
  run keep128_b0 BSMR_TILE_MIN_F32=128 BSMR_DIAG=8388608
done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r06n/*.json")):
    v=[json.loads(l) for l in open(f)]
    print(f.split('/')[-1], [round(d["ms_per_step"]*1e3,2) for d in v], v[0]["roofline"]["kernel"][:50])
PY
