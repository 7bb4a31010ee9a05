set -o pipefail
O=gpurun_out/j14
mkdir -p $O
export TMPDIR=/tmp
for pm in 16 12 8 6; do
BSMR_PIECE_MAX=$pm timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-vendor --cold-steps 0 > $O/C2_$pm.json 2>> $O/err.log &&
BSMR_PIECE_MAX=$pm timeout -k 10 300 python3 bench.py --config C3 --steps 30 --warmup 5 --no-cpu-baseline --no-vendor --cold-steps 0 > $O/C3_$pm.json 2>> $O/err.log &&
BSMR_PIECE_MAX=$pm timeout -k 10 300 python3 bench.py --config C5 --steps 50 --warmup 5 --no-cpu-baseline --no-vendor --cold-steps 0 > $O/C5u_$pm.json 2>> $O/err.log &&
BSMR_PIECE_MAX=$pm timeout -k 10 300 python3 tools/prof_sddmm.py --iters 10 --workload reddit_like --scale 0.25 > $O/C4q_$pm.json 2>> $O/err.log || exit 1
done
