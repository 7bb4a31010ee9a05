# multi-process rehearsal of bench.py --gpus 2 on one GPU (gloo; both ranks on cuda:0)
set -o pipefail
O=gpurun_out/j15
mkdir -p $O
export TMPDIR=/tmp
BSMR_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_g2.json 2> $O/bench_g2.err
