#!/bin/bash
# Round-3 first pass (through gpurun): smoke, the GPU suite (verbose: one line per test), the C2
# bench line, the C1 host-path line, and the drop-in binary's test-mode logs of Trefethen_20000
# (fixtures for the analyze_results.cpp test). Every GPU step has its own limit; the first failure
# ends the pass.
set -o pipefail
TAG=${1:-r03a}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*" >> "$OUT/steps.log"; }
step smoke && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
step pytest && timeout -k 10 1500 python3 -u -m pytest tests -x -v -m gpu --timeout 900 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
step bench && timeout -k 10 300 python3 bench.py > "$OUT/bench_C2.json" 2> "$OUT/bench_C2.err" &&
step C1 && timeout -k 10 300 python3 bench.py --config C1 > "$OUT/bench_C1.json" 2> "$OUT/bench_C1.err" &&
step testmode && timeout -k 10 300 python3 -c "
import sys; sys.path.insert(0, 'sddmm-gpu_amd')
from bsmr import synth
M, N, rp, ci = synth.SUITESPARSE_REBUILDS['Trefethen_20000']()
synth.write_mtx('/tmp/Trefethen_20000.mtx', M, N, rp, ci)" &&
mkdir -p "$OUT/testmode_Trefethen_20000" &&
timeout -k 10 300 ./sddmm-gpu_amd/bin/BSMR-sddmm -f /tmp/Trefethen_20000.mtx -t 1 -l "$OUT/testmode_Trefethen_20000/" > "$OUT/testmode.log" 2>&1
rc=$?
step "done rc=$rc"
echo "rc=$rc" > "$OUT/rc.txt"
exit $rc
