set -o pipefail
O=gpurun_out/j13
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-vendor > $O/C2.json 2>> $O/err.log &&
timeout -k 10 300 python3 bench.py --config C3 --steps 30 --warmup 5 --no-cpu-baseline --no-vendor --cold-steps 0 > $O/C3.json 2>> $O/err.log &&
timeout -k 10 300 python3 tools/trace_sddmm.py --workload cop20k_like --K 256 --dtype f16 > $O/trace_c3.json 2>> $O/err.log &&
timeout -k 10 300 python3 bench.py --config C5 --steps 50 --warmup 5 --no-cpu-baseline --no-vendor --cold-steps 0 > $O/C5u.json 2>> $O/err.log
