#!/bin/bash
# C4 at full size (reddit_like x1: 232,965 rows, ~232M stored entries, K=128 fp32): one global
# plan, the unsharded launch and the 1/2/4/8 row-panel shards timed one after another on this GPU
# (tools/shard_sim.py). A heartbeat file keeps the long plan build visibly alive.
set -o pipefail
O=gpurun_out/${1:-c4full}
mkdir -p $O
export TMPDIR=/tmp
(while true; do date >> $O/heartbeat; sleep 50; done) &
HB=$!
timeout -k 10 1000 python3 -u tools/shard_sim.py --workload reddit_like --scale 1.0 --iters 5 > $O/shard_c4.json 2> $O/shard_c4.err
rc=$?
kill $HB
echo "rc=$rc" > $O/rc.txt
exit $rc
