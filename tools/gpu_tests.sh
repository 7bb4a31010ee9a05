#!/bin/bash
# smoke() + the whole GPU suite (through gpurun): bash tools/gpu_tests.sh <tag>
set -o pipefail
TAG=${1:-tests}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 1000 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "rc=$rc" > "$OUT/rc.txt"
exit $rc
