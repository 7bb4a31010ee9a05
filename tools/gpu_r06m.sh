set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06m; mkdir -p $O
timeout -k 10 200 python3 tools/c2_union.py > $O/c2_union.json 2> $O/c2_union.err || exit 1
timeout -k 10 300 python3 tools/transpose_ab.py --reps 3 > $O/transpose_ab.json 2> $O/transpose_ab.err || exit 2
cat $O/c2_union.json; echo; cat $O/transpose_ab.json
