set -o pipefail
O=gpurun_out/j7
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for tm in 0 96 128 160 192 257; do
BSMR_TILE_MIN_F32=$tm timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-vendor --steps 100 > $O/C2_$tm.json 2>> $O/err.log || exit 1
BSMR_TILE_MIN_F32=$tm timeout -k 10 300 python3 tools/prof_sddmm.py --iters 10 --workload reddit_like --scale 0.25 > $O/C4q_$tm.json 2>> $O/err.log || exit 1
done
for tm in 0 32 64 128; do
BSMR_TILE_MIN_HALF=$tm timeout -k 10 300 python3 bench.py --config C3 --steps 30 --warmup 5 --no-cpu-baseline --no-vendor --cold-steps 0 > $O/C3_$tm.json 2>> $O/err.log || exit 1
BSMR_TILE_MIN_HALF=$tm timeout -k 10 300 python3 bench.py --config C5 --steps 50 --warmup 5 --no-cpu-baseline --no-vendor --cold-steps 0 > $O/C5u_$tm.json 2>> $O/err.log || exit 1
done
