set -o pipefail
mkdir -p gpurun_out/j1
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-vendor > gpurun_out/j1/bench_C2.json 2> gpurun_out/j1/bench_C2.err &&
timeout -k 10 300 python3 bench.py --config C3 --steps 50 --warmup 5 --no-cpu-baseline --no-vendor > gpurun_out/j1/bench_C3.json 2> gpurun_out/j1/bench_C3.err &&
bash tools/gpu_c4pmc.sh j1/c4pmc 0.25
