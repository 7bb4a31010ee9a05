#!/bin/bash
# One gpurun pass made of named steps, each under its own time limit, stopping at the first
# failure:   bash tools/gpu_steps.sh <tag> <step> [<step> ...]
# Outputs go to gpurun_out/<tag>/ (steps.log records the order and timing).
#   smoke                   __graft_entry__.smoke()
#   tests                   the whole pytest -m gpu suite (-v, per-test timeout)
#   tests:<a+b+...>         pytest -m gpu -k 'a or b or ...'
#   bench:<cfg>             bench.py line of one config (C1 C2 C3 C4 C4x1 C5u C5b C2k32 C2k512)
#   quick:<cfg>             the same without the CPU / vendor legs and PMC passes
#   pmc:<cfg>               the same without the CPU / vendor legs, with the in-run PMC traffic
#   sustained:<cfg>         quick, plus the busy-device time (--sustained: timing.sustained_*)
#   graph:<cfg>             quick, plus the timed steps replayed from one HIP graph (graph_replay)
#   rocprof:<cfg>           rocprofv3 --kernel-trace --stats of that config's bench (every traced
#                           launch a timed step)
#   strong:<scale>          bench's multi-GPU path on one GPU under torchrun (RCCL, world 1) with
#                           the strong_C4 block at that reddit-like scale
#   ss                      tools/suitesparse_compare.py (five rebuilt SuiteSparse matrices)
#   hybrid                  tools/hybrid_table.py (-t 1 logs of the five matrices + analyzer table)
#   ab:VAR:v1,v2:cfg1,cfg2  tools/ab_env.sh: alternating A/B of one BSMR_* knob (VAR without the
#                           prefix may list several, joined by '+') on ab_env.sh's configs
#   planab:<scale>:d1,d2,...  reddit-like plan build (tools/plan_time.py) under each BSMR_DIAG value
#                           in turn (permutation hash and clustering ms per run)
#   ablib:<variant.so>:cfg1,cfg2[:swap]   tools/ab_lib.sh: the in-tree library against a variant
#                           build (swap: the variant runs first in each pair)
#   driver                  exactly the driver's BENCH command (bench.py --gpus 1 --steps 20
#                           --warmup 5, every leg: PMC traffic, CPU baseline, vendor)
#   driverprof              rocprofv3 --kernel-trace --stats of exactly the driver's BENCH command
#                           (bench.py --gpus 1 --steps 20 --warmup 5; --pmc off: the in-run PMC
#                           children would run under the tracer too) + tools/rocprof_runs.py
#   guard                   tools/perf_guard.py --check profiles/perf_baseline.json: the 20
#                           published SuiteSparse points + C2-C5 against the committed baseline,
#                           rc 1 on any > 5 % loss (run after every layout-rule commit)
#   guard:record            the same points written as a new baseline (gpurun_out/<tag>/)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
log() { echo "[$(date +%T)] $*" >> "$OUT/steps.log"; }

cfg_args() {
    case "$1" in
        C1) echo "--config C1" ;;
        C2) echo "--config C2" ;;
        C2k32) echo "--config C2 --K 32" ;;
        C2k512) echo "--config C2 --K 512" ;;
        C3) echo "--config C3 --steps 50 --warmup 5" ;;
        C4) echo "--config C4 --steps 20 --warmup 3" ;;
        C4x1) echo "--config C4 --scale 1.0 --steps 20 --warmup 3 --cold-steps 0" ;;
        C5u) echo "--config C5 --mask uniform --steps 100 --warmup 10" ;;
        C5b) echo "--config C5 --mask block --steps 100 --warmup 10" ;;
        *) echo "unknown config $1" >&2; return 1 ;;
    esac
}
QUICK="--no-cpu-baseline --no-vendor --pmc off"

run_step() {
    local s=$1 name=${1%%:*} arg=${1#*:}
    local f=${s//[:\/ ]/_}
    log "start $s"
    case "$name" in
        smoke) timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
        tests)
            if [ "$arg" = "$s" ]; then
                timeout -k 10 1500 python3 -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
            else
                timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu -k "${arg//+/ or }" --timeout 600 --timeout-method thread > "$OUT/${f//+/_}.log" 2>&1
            fi ;;
        bench) timeout -k 10 900 python3 bench.py $(cfg_args "$arg") > "$OUT/bench_$arg.json" 2> "$OUT/bench_$arg.err" ;;
        quick) timeout -k 10 600 python3 bench.py $(cfg_args "$arg") $QUICK > "$OUT/quick_$arg.json" 2> "$OUT/quick_$arg.err" ;;
        sustained) timeout -k 10 600 python3 bench.py $(cfg_args "$arg") $QUICK --sustained > "$OUT/sustained_$arg.json" 2> "$OUT/sustained_$arg.err" ;;
        graph) timeout -k 10 600 python3 bench.py $(cfg_args "$arg") $QUICK --graph > "$OUT/graph_$arg.json" 2> "$OUT/graph_$arg.err" ;;
        pmc) timeout -k 10 600 python3 bench.py $(cfg_args "$arg") --no-cpu-baseline --no-vendor --pmc on > "$OUT/pmc_$arg.json" 2> "$OUT/pmc_$arg.err" ;;
        rocprof) timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$arg" -o run -- \
                     python3 bench.py $(cfg_args "$arg") $QUICK --no-split > "$OUT/rocprof_$arg.json" 2> "$OUT/rocprof_$arg.err" ;;
        strong) timeout -k 10 1000 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
                     --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --force-sharded \
                     --strong on --strong-scale "$arg" --no-vendor --pmc off > "$OUT/strong_$arg.json" 2> "$OUT/strong_$arg.err" ;;
        ss) timeout -k 10 1000 python3 -u tools/suitesparse_compare.py --out "$OUT/ss" > "$OUT/ss.log" 2>&1 ;;
        hybrid) timeout -k 10 1100 python3 -u tools/hybrid_table.py --run --out "$OUT/hybrid" > "$OUT/hybrid.log" 2>&1 ;;
        ab) IFS=: read -r _ var vals cfgs <<< "$s"
            timeout -k 10 1100 bash tools/ab_env.sh "$TAG/ab_${var//+/_}" "BSMR_${var//+/,BSMR_}" "${vals//,/ }" "${cfgs//,/ }" > "$OUT/$f.log" 2>&1 ;;
        ablib) IFS=: read -r _ so cfgs order <<< "$s"
            timeout -k 10 1100 bash tools/ab_lib.sh "$TAG/ablib_$(basename "$so" .so)${order:+_$order}" "$so" "${cfgs//,/ }" $order > "$OUT/$f.log" 2>&1 ;;
        planab) IFS=: read -r _ scale diags <<< "$s"
            for d in ${diags//,/ }; do
                BSMR_DIAG=$d timeout -k 10 300 python3 tools/plan_time.py --workload reddit_like --scale "$scale" --batches 16384 > "$OUT/plan_${scale}_$d.json" 2>> "$OUT/$f.log" || return $?
                python3 -c "import json; d=json.load(open('$OUT/plan_${scale}_$d.json')); r=list(d['runs'].values())[0]; print('scale $scale diag $d', r['row_reorder_ms'], r['rows_sha256'], r['num_clusters'], r['wall_s'])" >> "$OUT/planab_summary.txt"
            done ;;
        driver) timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/driver.json" 2> "$OUT/driver.err" ;;
        driverprof) timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_driver" -o run -- \
                     python3 bench.py --gpus 1 --steps 20 --warmup 5 --pmc off > "$OUT/driverprof.json" 2> "$OUT/driverprof.err" &&
                   python3 tools/rocprof_runs.py "$(ls "$OUT"/prof_driver/*/run_kernel_trace.csv "$OUT"/prof_driver/run_kernel_trace.csv 2>/dev/null | head -1)" > "$OUT/driverprof_runs.json" ;;
        guard)
            if [ "$arg" = "record" ]; then
                timeout -k 10 900 python3 -u tools/perf_guard.py --record "$OUT/perf_baseline.json" > "$OUT/guard_record.log" 2>&1
            else
                timeout -k 10 900 python3 -u tools/perf_guard.py --check profiles/perf_baseline.json --out "$OUT/guard.json" > "$OUT/guard.log" 2>&1
            fi ;;
        *) echo "unknown step $s" >&2; return 2 ;;
    esac
    local rc=$?
    log "end $s rc=$rc"
    return $rc
}

for s in "$@"; do
    run_step "$s" || { rc=$?; log "stopped at $s rc=$rc"; exit $rc; }
done
log "done"
