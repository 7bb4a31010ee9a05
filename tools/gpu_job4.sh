set -o pipefail
O=gpurun_out/j4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-vendor > $O/bench_C2.json 2> $O/bench_C2.err &&
timeout -k 10 300 python3 bench.py --config C3 --steps 50 --warmup 5 --no-cpu-baseline --no-vendor > $O/bench_C3.json 2> $O/bench_C3.err &&
for kb in 2048 1024 4096; do
BSMR_L2_RANGE_KB=$kb timeout -k 10 300 python3 tools/prof_sddmm.py --iters 10 --workload reddit_like --scale 0.25 > $O/c4q_$kb.json 2>> $O/c4q.err || exit 1
done &&
timeout -k 10 300 python3 tools/trace_sddmm.py --workload reddit_like --scale 0.25 > $O/trace_c4q.json 2> $O/trace_c4q.err
