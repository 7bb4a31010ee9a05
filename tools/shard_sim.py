#!/usr/bin/env python3
"""Row-panel sharding rehearsal on ONE GPU: one global BSMR plan, the cost-model
panel cuts for world = 1, 2, 4, 8, and each shard's SDDMM (bsmr_sddmm_panels: the row-block kernel
over that shard's own layout) timed alone on the whole GPU with HIP events, as rank r of an N-GPU
node would run it. Reports per-shard ms, the slowest shard (the job's step time), the imbalance
(max / mean) and the aggregate GFLOP/s = 2 nnz K / slowest; checks the union of the shards against
the unsharded launch (checkData rule). B broadcast time is not included (bench.py --gpus N
measures it over RCCL).

    python3 tools/shard_sim.py --workload reddit_like --scale 0.5 --K 128
    python3 tools/shard_sim.py --workload nips_like --copies 8   # bench --gpus 8 (C2 weak) rank by rank
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sddmm-gpu_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="reddit_like")
    ap.add_argument("--scale", type=float, default=None)
    ap.add_argument("--K", type=int, default=128)
    ap.add_argument("--dtype", default="f32", choices=["f32", "f16", "bf16"])
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--copies", type=int, default=1,
                    help="stack this many column-relabelled copies (bench.py's C2 weak scaling at "
                         "--gpus copies; synth.stack_copies) and shard over world = copies only")
    ap.add_argument("--rebalance", type=int, default=0,
                    help="rounds of measured-cost re-cutting (bsmr_plan_shard_rebalance, as "
                         "bench.py's global split does) after the model's cut")
    ap.add_argument("--local", action="store_true",
                    help="also time bench.py --shard local: contiguous original row panels of equal "
                         "stored entries, each on its own BSMR plan")
    args = ap.parse_args()
    import numpy as np
    import torch

    import bsmr
    import oracle_lib as O
    from bsmr import Plan, make_data, set_default_tuning, synth, tuning_from_env

    gen = getattr(synth, args.workload)
    M, N, rp, ci = gen(args.scale) if args.scale is not None else gen()
    if args.copies > 1:
        M, N, rp, ci = synth.stack_copies(M, N, rp, ci, args.copies)
        args.worlds = str(args.copies)
    K = args.K
    code = {"f32": bsmr.F32, "f16": bsmr.F16, "bf16": bsmr.BF16}[args.dtype]
    tdt = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}[args.dtype]
    t0 = time.perf_counter()
    set_default_tuning(tuning_from_env())  # BSMR_* A/B knobs (the library reads no env)
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3)
    plan_s = time.perf_counter() - t0
    print(f"plan {plan_s:.1f} s", file=sys.stderr, flush=True)
    nnz = len(ci)
    dA = torch.from_numpy(make_data(M * K)).cuda().to(tdt)
    dB = torch.from_numpy(make_data(N * K)).cuda().to(tdt)
    dP = torch.zeros(nnz, dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream()
    s = stream.cuda_stream
    flops = 2.0 * nnz * K

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.iters):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.iters

    t0 = time.perf_counter()
    plan.sddmm(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), stream=s, dtype=code)
    torch.cuda.synchronize()
    layout_s = time.perf_counter() - t0  # the first call builds the row-block layout
    full_ms = timed(lambda: plan.sddmm(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), stream=s,
                                       dtype=code))
    P_full = dP.cpu().numpy()
    out = {"workload": args.workload, "scale": args.scale, "M": M, "N": N, "nnz": nnz, "K": K,
           "dtype": args.dtype, "plan_build_s": round(plan_s, 2),
           "first_call_s": round(layout_s, 2), "plan_stats": plan.stats(),
           "unsharded": {"ms": round(full_ms, 5), "GFLOP/s": round(flops / full_ms / 1e6, 1)},
           "worlds": {}}
    bo = plan.array("blockOffsets").astype(np.int64)
    so = plan.array("sparseValueOffsets").astype(np.int64)
    for world in [int(w) for w in args.worlds.split(",")]:
        shards = [plan.shard(K, r, world, code) for r in range(world)]
        history = []
        for it in range(args.rebalance + 1):
            dP.fill_(float("nan"))
            ms = []
            for p0, p1 in shards:
                ms.append(timed(lambda: plan.sddmm_panels(dA.data_ptr(), dB.data_ptr(), K,
                                                           dP.data_ptr(), p0, p1, stream=s,
                                                           dtype=code)))
            history.append({"cuts": [a for a, _ in shards] + [shards[-1][1]],
                            "shard_ms": [round(x, 5) for x in ms], "step_ms": round(max(ms), 5),
                            "imbalance": round(max(ms) / (sum(ms) / len(ms)), 3)})
            if it == args.rebalance or world == 1:
                break
            cuts = plan.shard_rebalance(K, world, history[-1]["cuts"], ms, code)
            shards = list(zip(cuts[:-1], cuts[1:]))
        best = min(range(len(history)), key=lambda i: history[i]["step_ms"])
        if best != len(history) - 1:  # the outputs below come from the fastest cut
            c = history[best]["cuts"]
            shards = list(zip(c[:-1], c[1:]))
            dP.fill_(float("nan"))
            ms = [timed(lambda: plan.sddmm_panels(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(),
                                                  p0, p1, stream=s, dtype=code))
                  for p0, p1 in shards]
        P = dP.cpu().numpy()
        slow = max(ms)
        out["worlds"][world] = {
            "rebalance_history": history,
            "shards": shards, "shard_ms": [round(x, 5) for x in ms],
            "shard_tiles": [int(bo[b] - bo[a]) for a, b in shards],
            "shard_residual": [int(so[b] - so[a]) for a, b in shards],
            "step_ms": round(slow, 5), "imbalance": round(slow / (sum(ms) / len(ms)), 3),
            "aggregate_GFLOP/s": round(flops / slow / 1e6, 1),
            "unwritten": int(np.isnan(P).sum()),
            "checkData_errors_vs_unsharded": O.check_data(P_full, P)}
        print(json.dumps({world: out["worlds"][world]}), file=sys.stderr, flush=True)
    if args.local:
        from bsmr import dist as D
        rp64 = np.asarray(rp, dtype=np.int64)
        for world in [int(w) for w in args.worlds.split(",")]:
            ms, cl = [], []
            for r in range(world):
                r0, r1 = D.row_range_cut(rp64, r, world)
                e0, e1 = int(rp64[r0]), int(rp64[r1])
                lp = Plan(r1 - r0, N, (rp64[r0:r1 + 1] - e0).astype(np.uint32),
                          np.ascontiguousarray(np.asarray(ci)[e0:e1], dtype=np.uint32),
                          alpha=0.3, delta=0.3)
                a_loc = dA[r0 * K:r1 * K].contiguous()
                p_loc = torch.zeros(e1 - e0, dtype=torch.float32, device="cuda")
                ms.append(timed(lambda: lp.sddmm(a_loc.data_ptr(), dB.data_ptr(), K,
                                                 p_loc.data_ptr(), stream=s, dtype=code)))
                cl.append(O.check_data(P_full[e0:e1], p_loc.cpu().numpy()))
                del lp
            slow = max(ms)
            out["worlds"][f"local{world}"] = {
                "shard_ms": [round(x, 5) for x in ms], "step_ms": round(slow, 5),
                "imbalance": round(slow / (sum(ms) / len(ms)), 3),
                "aggregate_GFLOP/s": round(flops / slow / 1e6, 1),
                "checkData_errors_vs_unsharded": int(sum(cl))}
            print(json.dumps({f"local{world}": out["worlds"][f"local{world}"]}), file=sys.stderr,
                  flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
