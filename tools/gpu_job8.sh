set -o pipefail
O=gpurun_out/j8
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/trace_sddmm.py > $O/trace_c2.json 2> $O/err.log &&
BSMR_LAYOUT_ROWBLOCK=1 timeout -k 10 300 python3 tools/trace_sddmm.py --workload reddit_like --scale 0.25 > $O/trace_c4q.json 2>> $O/err.log &&
for lds in 144 120 96 72; do
timeout -k 10 300 python3 tools/prof_sddmm.py --iters 20 --lds-kb $lds > $O/c2_lds$lds.json 2>> $O/err.log || exit 1
done
