set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ak; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu -k "parity or staged or out_packed or item_sched or colblocks or fullsize or plan_check" --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 1100 bash tools/ab_lib.sh r06ak/ablib sddmm-gpu_amd/lib_exp/libbsmr_amd.so "C3 M14k256 M15k64 C2" > $O/ablib.log 2>&1 || { tail -5 $O/ablib.log; exit 2; }
python3 - <<'PY'
import collections
d=collections.defaultdict(lambda: collections.defaultdict(list))
for l in open("gpurun_out/r06ak/ablib/summary.txt"):
    c,v,t=l.split(); d[c][v].append(float(t)*1e3)
for c in d: print(c, {v: [round(x,2) for x in d[c][v]] for v in d[c]})
PY
