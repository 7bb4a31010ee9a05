set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06aj; mkdir -p $O
timeout -k 10 1100 bash tools/ab_lib.sh r06aj/ablib_roll sddmm-gpu_amd/lib_exp/libbsmr_amd.so "C2 C2k32 C2k512 C3 M15k32 M14k256" > $O/ablib.log 2>&1 || { tail -5 $O/ablib.log; exit 2; }
python3 - <<'PY'
import collections
d=collections.defaultdict(lambda: collections.defaultdict(list))
for l in open("gpurun_out/r06aj/ablib_roll/summary.txt"):
    c,v,t=l.split(); d[c][v].append(float(t)*1e3)
for c in d: print(c, {v: [round(x,2) for x in d[c][v]] for v in d[c]})
PY
