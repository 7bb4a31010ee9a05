#!/usr/bin/env python3
"""C4 (reddit-like) memory floor and piece census.

Builds the bench's C4 plan (reddit_like x scale, fp32 K = 128), times the product launch, dumps its
row-block layout (bsmr_debug_rb_pieces) and replays exactly that layout's data stream on
tools/ubench/c4floor.hip — the same items in the same pair schedule, the same A row-block images
by LDS-DMA, the same column-run pieces (descriptor, 512-byte B row, entry metadata), no LDS reads,
no FMA, no stores. The replay's time is the floor of this stream; product / floor says how much of
the launch is anything but moving these bytes. The census: pieces by entry count and by the stored-
entry count (degree) of their column.

    hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/ubench/libc4floor.so tools/ubench/c4floor.hip
    python3 tools/c4_floor.py --scale 1.0 --iters 10 > c4_floor.json
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sddmm-gpu_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--lib", default=os.path.join(ROOT, "tools", "ubench", "libc4floor.so"))
    args = ap.parse_args()
    import torch

    import bsmr
    from bsmr import Plan, make_data, synth

    t0 = time.perf_counter()
    M, N, rp, ci = synth.reddit_like(args.scale)
    K, nnz = 128, len(ci)
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3)
    dev = torch.device("cuda", 0)
    dA = torch.from_numpy(make_data(M * K)).to(dev)
    dB = torch.from_numpy(make_data(N * K)).to(dev)
    dP = torch.zeros(nnz, dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream

    def timed(fn, n):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(n):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n

    prod_ms = timed(lambda: plan.sddmm(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), stream=sp), args.iters)
    st = plan.stats()
    L = bsmr.lib()
    L.bsmr_debug_rb_items.argtypes = [C.c_void_p, C.c_uint32, C.c_int, C.c_void_p, C.POINTER(C.c_uint64)]
    L.bsmr_debug_rb_pieces.argtypes = [C.c_void_p, C.c_uint32, C.c_int, C.c_void_p, C.POINTER(C.c_uint64)]
    n = C.c_uint64()
    L.bsmr_debug_rb_items(plan.h, K, 0, None, C.byref(n))
    hdr = np.zeros(n.value, np.uint32)
    L.bsmr_debug_rb_items(plan.h, K, 0, hdr.ctypes.data, C.byref(n))
    RB, NT, nslots, rowBytes = (int(x) for x in hdr[:4])
    L.bsmr_debug_rb_pieces(plan.h, K, 0, None, C.byref(n))
    buf = np.zeros(n.value, np.uint32)
    L.bsmr_debug_rb_pieces(plan.h, K, 0, buf.ctypes.data, C.byref(n))
    ni, npc = int(buf[0]), int(buf[1])
    items = buf[2:2 + 4 * ni].reshape(ni, 4)
    iend = buf[2 + 4 * ni:2 + 5 * ni]
    pieces = buf[2 + 5 * ni:2 + 5 * ni + 2 * npc].reshape(npc, 2)
    plen = (pieces[:, 1] >> 22) + 1
    pcol = pieces[:, 1] & 0x3FFFFF
    entries = int(plen.sum())
    deg = np.bincount(np.asarray(ci, np.int64), minlength=N)
    out = {"workload": f"reddit_like x{args.scale} fp32 K={K}", "M": M, "N": N, "nnz": nnz,
           "layout": {"rows_per_block": RB, "threads": NT, "item_slots": ni, "pieces": npc,
                      "entries_in_pieces": entries, "row_bytes": rowBytes,
                      "pairs": bool(st["rb_pairs"] & 4), "batches": bool(st["rb_batches"] & 4)},
           "product_ms": round(prod_ms, 4),
           "product_tflops": round(2.0 * nnz * K / (prod_ms * 1e-3) / 1e12, 3)}
    # census: pieces by length, and pieces / entries by their column's degree (log2 buckets)
    out["census"] = {
        "pieces_by_len": {int(k): int(v) for k, v in zip(*np.unique(plen, return_counts=True))},
        "entries_per_piece": round(entries / npc, 3)}
    dbin = np.floor(np.log2(np.maximum(deg[pcol], 1))).astype(int)
    by = {}
    for b in np.unique(dbin):
        m = dbin == b
        by[f"deg 2^{b}..2^{b + 1}"] = {"pieces": int(m.sum()), "entries": int(plen[m].sum()),
                                       "entries_per_piece": round(float(plen[m].mean()), 3),
                                       "columns": int(((np.floor(np.log2(np.maximum(deg, 1))) == b) & (deg > 0)).sum())}
    out["census"]["by_column_degree"] = by
    # bytes of the stream (L2 -> CU): A images (pairs stage the second item only on a new block),
    # one B row per piece, 8 B descriptor per piece, 4 B metadata per entry
    stage_blocks = (RB * rowBytes + 1023) // 1024
    real = ~((items[:, 1] == items[:, 2]) & (items[:, 3] == iend))
    pos = np.arange(ni)
    second = (pos // 8) % 2 == 1
    first_rb = items[np.where(second, pos - 8, pos), 0]
    staged = real & (~second | (items[:, 0] != first_rb))
    a_bytes = int(staged.sum()) * stage_blocks * 1024
    b_bytes = npc * rowBytes
    meta_bytes = 8 * npc + 4 * entries
    out["stream_bytes"] = {"A_images": a_bytes, "B_rows": b_bytes, "piece_meta": meta_bytes,
                           "total": a_bytes + b_bytes + meta_bytes,
                           "items_staged": int(staged.sum())}
    # the replay
    if os.path.exists(args.lib):
        F = C.CDLL(args.lib)
        F.c4floor_launch.argtypes = [C.c_void_p] * 7 + [C.c_uint] * 4 + [C.c_void_p] * 2
        t_items = torch.from_numpy(items.astype(np.int32)).to(dev)
        t_iend = torch.from_numpy(iend.astype(np.int32)).to(dev)
        t_pcs = torch.from_numpy(pieces.astype(np.int32)).to(dev)
        t_meta = torch.zeros(max(entries, 1) + 64, dtype=torch.int32, device=dev)
        t_rows = torch.from_numpy(plan.array("reorderedRows").astype(np.int32)).to(dev)
        sink = torch.zeros(1024, dtype=torch.float32, device=dev)

        def floor():
            rc = F.c4floor_launch(dA.data_ptr(), dB.data_ptr(), t_items.data_ptr(), t_iend.data_ptr(),
                                  t_pcs.data_ptr(), t_meta.data_ptr(), t_rows.data_ptr(),
                                  st["num_reordered_rows"], RB, ni, stage_blocks, sink.data_ptr(), sp)
            assert rc == 0
        floor_ms = timed(floor, args.iters)
        out["floor_ms"] = round(floor_ms, 4)
        out["product_over_floor"] = round(prod_ms / floor_ms, 3)
        out["floor_stream_TBps"] = round(out["stream_bytes"]["total"] / (floor_ms * 1e-3) / 1e12, 2)
        out["product_stream_TBps"] = round(out["stream_bytes"]["total"] / (prod_ms * 1e-3) / 1e12, 2)
    else:
        out["floor_ms"] = None
        out["note"] = f"{args.lib} not built"
    out["wall_s"] = round(time.perf_counter() - t0, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
