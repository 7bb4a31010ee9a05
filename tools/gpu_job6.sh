set -o pipefail
O=gpurun_out/j6
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu -k "shard" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python3 tools/shard_sim.py --workload reddit_like --scale 0.25 > $O/shard_c4q.json 2> $O/shard_c4q.err &&
timeout -k 10 600 python3 tools/shard_sim.py --workload reddit_like --scale 0.5 > $O/shard_c4h.json 2> $O/shard_c4h.err
