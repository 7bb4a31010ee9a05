set -o pipefail
O=gpurun_out/j2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu -k "shard or batch or rowblock or layout" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-vendor > $O/bench_C2.json 2> $O/bench_C2.err &&
timeout -k 10 300 python3 bench.py --config C3 --steps 50 --warmup 5 --no-cpu-baseline --no-vendor > $O/bench_C3.json 2> $O/bench_C3.err &&
timeout -k 10 300 python3 tools/prof_sddmm.py --iters 10 --workload reddit_like --scale 0.25 > $O/c4q.json 2> $O/c4q.err &&
timeout -k 10 600 python3 tools/shard_sim.py --workload reddit_like --scale 0.25 > $O/shard_c4q.json 2> $O/shard_c4q.err
