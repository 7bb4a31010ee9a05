// Memory floor of a row-block launch's own data stream: the exact items,
// row blocks and column-run pieces of a plan's row-block layout (bsmr_debug_rb_pieces), replayed
// with the product kernel's geometry for 512-byte rows (1024 threads, G = 4 lanes per row-group,
// 8 chunks of 16 B per lane) and its pair schedule (workgroup j runs list positions 2j and
// 2j + 1 of its XCD, the second item staged only when its row block differs) — but with no LDS
// reads, no FMA and no result: per item the A image by LDS-DMA, then per piece its descriptor,
// its B row (512 B) and its entries' metadata, one piece ahead in flight per row-group.
// What this launch takes is the time of the gathers alone; the product launch on the same layout
// can not be faster than it.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o libc4floor.so c4floor.hip
#include <hip/hip_runtime.h>

#include <cstdint>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned u32;

struct FloorArgs {
    const char* A;        // M x 512 B rows
    const char* B;        // N x 512 B rows
    const uint4* items;   // {row block, tile begin, tile end, piece begin}
    const u32* itemEnd;   // piece end
    const uint2* pieces;  // {first entry, column | (len - 1) << 22}
    const u32* meta;      // entry metadata (4 B per entry)
    const u32* rows;      // reordered rows
    u32 R, RB, nItems, stageBlocks;
    float* sink;          // never written in practice (keeps the loads)
};

constexpr u32 NT = 1024, NW = 16, G = 4, NG = NT / G, NC = 8, RBY = 512;

__device__ __forceinline__ u32 lds_addr(const char* l) {
    return __builtin_amdgcn_readfirstlane(static_cast<u32>(
        reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const char*)l)));
}

__device__ __forceinline__ void dma16(const char* g, const u32 m0) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m0)
                 : "memory", "m0");
}

// stage the item's row block: every wave issues its 1 KiB blocks of the image (2 rows each)
__device__ __forceinline__ void stage(const FloorArgs& a, char* As, const u32 q0, const u32 ws,
                                      const u32 lane) {
    const u32 half = lane >> 5, chunk = lane & 31;
    for (u32 b = ws; b < a.stageBlocks; b += NW) {
        const u32 lr = 2 * b + half, q = q0 + lr;
        const u32 row = (lr < a.RB && q < a.R) ? a.rows[q] : a.rows[0];
        dma16(a.A + static_cast<size_t>(row) * RBY + 16 * chunk, lds_addr(As) + 1024 * b);
    }
}

__global__ __launch_bounds__(NT) void k_floor(FloorArgs a) {
    extern __shared__ __attribute__((aligned(16))) char As[];
    const u32 tid = threadIdx.x, lane = tid & 63, ws = __builtin_amdgcn_readfirstlane(tid >> 6);
    const u32 gr = tid / G, sub = tid % G;
    const u32 x = blockIdx.x % 8, i0 = (blockIdx.x / 8) * 16 + x;
    float acc = 0.f;
    u32 prev_rb = 0xFFFFFFFFu;
    for (u32 k = 0; k < 2; ++k) {
        const u32 idx = i0 + 8 * k;
        if (idx >= a.nItems) break;
        const uint4 it = a.items[idx];
        const u32 pend = a.itemEnd[idx];
        if (it.y == it.z && it.w == pend) break;  // padding (a suffix of each list)
        const u32 rb = __builtin_amdgcn_readfirstlane(it.x);
        if (rb != prev_rb) {
            __syncthreads();
            stage(a, As, rb * a.RB, ws, lane);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            prev_rb = rb;
        }
        // pieces [it.w, pend): row-group gr takes it.w + gr, + NG, ...; one piece ahead in flight
        u32 p = it.w + gr;
        f4 bv[NC];
        u32 mm[4];
        auto fetch = [&](const u32 pi) {
            const uint2 d = a.pieces[pi];
            const u32 col = d.y & 0x3FFFFFu, len = (d.y >> 22) + 1;
            const char* bp = a.B + static_cast<size_t>(col) * RBY + 16 * sub;
#pragma unroll
            for (u32 f = 0; f < NC; ++f) bv[f] = *reinterpret_cast<const f4*>(bp + 16 * G * f);
#pragma unroll
            for (u32 m = 0; m < 4; ++m) mm[m] = G * m + sub < len ? a.meta[d.x + G * m + sub] : 0u;
        };
        if (p < pend) fetch(p);
        while (p < pend) {
            f4 cur[NC];
#pragma unroll
            for (u32 f = 0; f < NC; ++f) cur[f] = bv[f];
            const u32 m0 = mm[0] ^ mm[1] ^ mm[2] ^ mm[3];
            p += NG;
            if (p < pend) fetch(p);
#pragma unroll
            for (u32 f = 0; f < NC; ++f) acc += cur[f].x;
            acc += __builtin_bit_cast(float, m0 & 0x3F7FFFFFu);
        }
    }
    if (acc == -1234.5f) a.sink[tid] = acc;  // never: keeps every load
}

extern "C" int c4floor_launch(const void* A, const void* B, const void* items, const void* itemEnd,
                              const void* pieces, const void* meta, const void* rows, unsigned R,
                              unsigned RB, unsigned nItems, unsigned stageBlocks, void* sink,
                              void* stream) {
    FloorArgs a;
    a.A = static_cast<const char*>(A);
    a.B = static_cast<const char*>(B);
    a.items = static_cast<const uint4*>(items);
    a.itemEnd = static_cast<const u32*>(itemEnd);
    a.pieces = static_cast<const uint2*>(pieces);
    a.meta = static_cast<const u32*>(meta);
    a.rows = static_cast<const u32*>(rows);
    a.R = R;
    a.RB = RB;
    a.nItems = nItems;
    a.stageBlocks = stageBlocks;
    a.sink = static_cast<float*>(sink);
    const u32 grid = (nItems + 1) / 2;
    hipLaunchKernelGGL(k_floor, dim3(grid), dim3(NT), 160 * 1024, static_cast<hipStream_t>(stream), a);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
