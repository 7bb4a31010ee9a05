set -o pipefail
O=gpurun_out/j3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/trace_sddmm.py --workload reddit_like --scale 0.25 > $O/trace_c4q.json 2> $O/trace_c4q.err &&
timeout -k 10 300 python3 tools/prof_sddmm.py --iters 10 --workload reddit_like --scale 0.25 > $O/c4q_order0.json 2> $O/c4q.err &&
BSMR_PIECE_ORDER=1 timeout -k 10 300 python3 tools/prof_sddmm.py --iters 10 --workload reddit_like --scale 0.25 > $O/c4q_order1.json 2>> $O/c4q.err &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-vendor > $O/bench_C2.json 2> $O/bench_C2.err &&
timeout -k 10 600 python3 tools/shard_sim.py --workload reddit_like --scale 0.25 > $O/shard_c4q.json 2> $O/shard_c4q.err
