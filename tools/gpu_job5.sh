set -o pipefail
O=gpurun_out/j5
mkdir -p $O
export TMPDIR=/tmp
for cfg in "144 2048" "72 2048" "72 3072" "72 1536" "144 3072"; do
set -- $cfg
BSMR_L2_RANGE_KB=$2 timeout -k 10 300 python3 tools/prof_sddmm.py --iters 10 --workload reddit_like --scale 0.25 --lds-kb $1 > $O/c4q_$1_$2.json 2>> $O/c4q.err || exit 1
done &&
for lds in 72 96; do
timeout -k 10 300 python3 tools/prof_sddmm.py --iters 10 --workload cop20k_like --K 256 --dtype f16 --lds-kb $lds > $O/c3_$lds.json 2>> $O/c3.err || exit 1
done
