set -o pipefail
O=gpurun_out/k32b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for K in 32 64 128; do timeout -k 10 300 python3 bench.py --K $K --steps 100 --no-cpu-baseline --no-vendor --cold-steps 0 > $O/C2_K$K.json 2>> $O/err.log || exit 1; done
timeout -k 10 300 python3 bench.py --config C5 --K 64 --steps 50 --warmup 5 --no-cpu-baseline --no-vendor --cold-steps 0 > $O/C5u_K64.json 2>> $O/err.log
