set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c; mkdir -p $O
for t in 4 2; do
BSMR_PTILE_TPI=$t timeout -k 10 300 python3 tools/trace_sddmm.py --workload dlmc_like --mask block --K 512 --dtype bf16 --waves-per-wg 1 --dump $O/trace_tpi$t.npy > $O/trace_tpi$t.json 2> $O/trace_tpi$t.err || exit 2
done
BSMR_PTILE=0 timeout -k 10 300 python3 tools/trace_sddmm.py --workload dlmc_like --mask block --K 512 --dtype bf16 --waves-per-wg 8 --dump $O/trace_dense.npy > $O/trace_dense.json 2> $O/trace_dense.err || exit 3
cat $O/*.json
