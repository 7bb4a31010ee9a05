// sddmm.hip — the SDDMM launch over a BSMR plan (gfx950, wave64, MFMA).
//
// One launch, one wave per work item (64-thread workgroups), two item kinds:
//   * dense tile {panel, tile}: 4*K/16 `v_mfma_f32_16x16x4_f32` (exact fp32; gfx950 has no TF32).
//     Lane l holds A[row l&15][16kk + 4(l>>4) + e] and B[col l&15][same k]; instruction e of step
//     kk sums k = 16kk + 4g + e over the four lane groups g, so every k is covered once.
//     Accumulator lane l, reg r = D[4(l>>4)+r][l&15], scattered through blockValues
//     (replaces sddmm_gpu_dense_block_m16n16k8_*, sddmmKernel.cu:213-351, 355-488).
//   * residual slot {e0, e1} of the column-major residual list: G lanes per entry, each lane one
//     16-byte piece of A[row] and of B[col] per K/(4G) step, U entries in flight per lane, xor
//     shuffle reduction (replaces sddmm_gpu_sparse_block_2_2threadOneData_shuffle,
//     sddmmKernel.cu:1994-2104). Entries are ordered by (col % 8, col): consecutive entries
//     share their B column, and slot s is bucket s % 8, so under the round-robin block->XCD
//     dispatch each XCD's L2 serves 1/8 of B plus the (small) A gather.
// The reference launches a panels x ceil(maxBlocks/4) dense grid plus a second kernel on another
// stream; here both parts are one balanced grid with no idle blocks.
// bsmr_sddmm_panels (row-panel shards) uses the panel-major residual items instead, with the
// panel's A rows staged in LDS.
#include <algorithm>
#include <type_traits>
#include <cmath>
#include <vector>

#include "common.hpp"
#include "plan.hpp"

namespace bsmr {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct SddmmArgs {
    const float* A;
    const float* B;
    float* P;
    // dense tiles [d0, d0 + nd) (one tile per wave)
    u32 d0, nd;
    const u32* tileRows;
    const u32* rows;
    u32 R, N, K;
    const u32* denseCols;
    const u32* blockValues;
    // column-major residual slots (full launch)
    const uint2* slots;
    u32 nslots;
    const u32* cmRow;
    const u32* cmCol;
    const u32* cmOut;
    // panel-major residual items (panel ranges)
    const uint4* ritems;
    u32 r0, nr;
    const u32* sparseValues;
    const u32* sparseRel;
    const u32* sparseCol;
    u32 diag;  // profiling ablations (BSMR_DIAG); always 0 in normal use
    unsigned long long* trace;  // BSMR_DIAG & 32: per-wave {start, mid, end, hw id}; else null
    // batched launch (grid.y = batch b): A += b * bA, B += b * bB, P += b * bP (elements)
    unsigned long long bA, bB, bP;
};

// debug timeline (BSMR_DIAG & 32 only): wave start / mid / end in s_memrealtime ticks (100 MHz)
// and the wave's XCC id << 32 | HW_ID register
__device__ __forceinline__ unsigned long long rtime(const void* on) {
    return on ? __builtin_amdgcn_s_memrealtime() : 0ull;
}
__device__ __forceinline__ void trace_wave(unsigned long long* tr, u32 slot, unsigned long long t0,
                                           unsigned long long tm, unsigned long long td = 0) {
    if (tr && __lane_id() == 0) {
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        const u32 xcc = __builtin_amdgcn_s_getreg(0xF814);  // HW_REG_XCC_ID, 32 bits
        tr[4ull * slot + 0] = t0;
        tr[4ull * slot + 1] = tm;
        tr[4ull * slot + 2] = t1;
        tr[4ull * slot + 3] = (static_cast<unsigned long long>(xcc) << 60) | (td ? td : tm);
    }
}

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ float dot4(f32x4 a, f32x4 b) {
    return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
}

// ---- one dense tile, K = KT (KT = 0: runtime K, multiple of 16). The tile's 16 A-row indices
// (tileRows), its 16 columns and its 256 output indices depend only on the tile id, so the wave
// has two dependent memory round trips: metadata, then A/B.
template <int KT>
__device__ __forceinline__ void dense_tile(const SddmmArgs& a, const u32 tile) {
    const u32 K = KT > 0 ? KT : a.K;
    const u32 l = __lane_id(), rr = l & 15, g = l >> 4;
    const u32 row = a.tileRows[tile * 16 + rr];
    const u32 c = a.denseCols[tile * 16 + rr];
    const u32* bvals = a.blockValues + static_cast<size_t>(tile) * 256 + 64 * g + rr;
    u32 idx[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) idx[r] = bvals[16 * r];
    const bool rvalid = row != NULLV;
    const bool cvalid = c < a.N;
    const float* arow = a.A + static_cast<size_t>(rvalid ? row : 0) * K + 4 * g;
    const float* bcol = a.B + static_cast<size_t>(cvalid ? c : 0) * K + 4 * g;
    f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};  // two chains halve the MFMA dependency
    if constexpr (KT > 0) {
        // chunks of at most 4 k-steps (64 k): 8 float4 = 32 VGPRs of operands in flight, so the
        // kernel fits 64 VGPRs (8 waves per SIMD)
        constexpr int NK = KT / 16;
        constexpr int CH = NK < 4 ? NK : 4;
#pragma unroll
        for (int k0 = 0; k0 < NK; k0 += CH) {
            f32x4 av[CH], bv[CH];
#pragma unroll
            for (int kk = 0; kk < CH; ++kk) {
                av[kk] = rvalid ? ld4(arow + 16 * (k0 + kk)) : f32x4{0, 0, 0, 0};
                bv[kk] = cvalid ? ld4(bcol + 16 * (k0 + kk)) : f32x4{0, 0, 0, 0};
            }
#pragma unroll
            for (int kk = 0; kk < CH; ++kk) {
                f32x4& acc = (kk & 1) ? acc1 : acc0;
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kk].x, bv[kk].x, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kk].y, bv[kk].y, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kk].z, bv[kk].z, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kk].w, bv[kk].w, acc, 0, 0, 0);
            }
        }
    } else {
        for (u32 k = 0; k < K; k += 16) {
            const f32x4 av = rvalid ? ld4(arow + k) : f32x4{0, 0, 0, 0};
            const f32x4 bv = cvalid ? ld4(bcol + k) : f32x4{0, 0, 0, 0};
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bv.x, acc0, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, bv.y, acc0, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, bv.z, acc0, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, bv.w, acc0, 0, 0, 0);
        }
    }
    const f32x4 acc = acc0 + acc1;
#pragma unroll
    for (int r = 0; r < 4; ++r)
        if (idx[r] != NULLV && (!(a.diag & 1) || acc[r] == -1234.5f)) a.P[idx[r]] = acc[r];
}

template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
    for (int o = G / 2; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// DPP helpers on 16-lane rows (VALU only, no LDS crossbar)
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                                 CTRL, 0xF, 0xF, false));
}
// sum over the 16 lanes of a row, every lane gets the total
__device__ __forceinline__ float row_sum16(float v) {
    v += dppf<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dppf<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dppf<0x141>(v);  // row_half_mirror
    v += dppf<0x140>(v);  // row_mirror
    return v;
}
// value of lane N of the row, in every lane of the row (row_newbcast, gfx90a+)
template <int N>
__device__ __forceinline__ u32 row_bcast(u32 v) {
    return static_cast<u32>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x150 + N, 0xF, 0xF,
                                                         false));
}

template <int W>
struct vec;
template <>
struct vec<4> {
    typedef float __attribute__((ext_vector_type(4))) t;
};
template <>
struct vec<2> {
    typedef float __attribute__((ext_vector_type(2))) t;
};
template <>
struct vec<1> {
    typedef float t;
};
template <int W>
__device__ __forceinline__ float vdot(typename vec<W>::t a, typename vec<W>::t b) {
    if constexpr (W == 4)
        return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
    else if constexpr (W == 2)
        return a.x * b.x + a.y * b.y;
    else
        return a * b;
}

// ---- column-major residual slot (K = KT known). One 16-lane row per entry: lane s holds the
// W-float pieces s, s+16, ... of A[row] and B[col]. Each row takes a contiguous share of the
// slot's entries (sorted by column); per batch of 16 entries the row loads the metadata once
// (one entry per lane) and broadcasts entry i with row_newbcast:i. U entries are in flight per
// lane; the B pieces are re-loaded only when the column changes (a column run costs one B read);
// the 16-lane dot-product reduction is four DPP adds.
template <int KT>
__device__ __forceinline__ void residual_cm(const SddmmArgs& a, const uint2 sl) {
    constexpr int W = KT >= 64 ? 4 : KT / 16;
    constexpr int NF = KT / (16 * W);
    constexpr int U = NF >= 4 ? 1 : 4 / NF;  // <= 64 VGPRs: 8 waves per SIMD
    typedef typename vec<W>::t vt;
    const u32 l = __lane_id(), sub = l & 15, grp = l >> 4;
    const u32 n = sl.y - sl.x;
    const u32 share = (n + 3) / 4;
    const u32 gs = sl.x + min(grp * share, n), ge = sl.x + min(grp * share + share, n);
    u32 curc = NULLV;
    vt bcur[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f) bcur[f] = vt{};
    for (u32 base = gs; base < ge; base += 16) {
        const u32 e = base + sub;
        const bool okm = e < ge;
        const u32 mrow = okm ? a.cmRow[e] : 0u;
        const u32 mcol = okm ? a.cmCol[e] : NULLV;
        const u32 mout = okm ? a.cmOut[e] : 0u;
        const u32 nb = min(16u, ge - base);
#pragma unroll
        for (int i0 = 0; i0 < 16; i0 += U) {
            if (static_cast<u32>(i0) >= nb) break;
            vt av[U][NF], bv[U][NF];
            u32 cc[U], oo[U];
            bool ok[U], chg[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                constexpr int dummy = 0;
                (void)dummy;
                u32 r;
                switch (i0 + u) {  // compile-time lane index after unrolling
#define BSMR_B(I)                    \
    case I:                          \
        r = row_bcast<I>(mrow);      \
        cc[u] = row_bcast<I>(mcol);  \
        oo[u] = row_bcast<I>(mout);  \
        break;
                    BSMR_B(0) BSMR_B(1) BSMR_B(2) BSMR_B(3) BSMR_B(4) BSMR_B(5) BSMR_B(6) BSMR_B(7)
                    BSMR_B(8) BSMR_B(9) BSMR_B(10) BSMR_B(11) BSMR_B(12) BSMR_B(13) BSMR_B(14)
                    BSMR_B(15)
#undef BSMR_B
                    default:
                        r = 0;
                        cc[u] = NULLV;
                        oo[u] = 0;
                }
                ok[u] = static_cast<u32>(i0 + u) < nb;
                const u32 prev = u ? cc[u - 1] : curc;
                chg[u] = ok[u] && cc[u] != prev;
                // a.diag (profiling ablations only; 0 in every real launch): 2 = A row 0, 4 = B col 0
                const u32 ar = (a.diag & 2) ? 0u : (ok[u] ? r : 0u);
                const float* ap = a.A + static_cast<size_t>(ar) * KT + W * sub;
#pragma unroll
                for (int f = 0; f < NF; ++f)
                    av[u][f] = *reinterpret_cast<const vt*>(ap + 16 * W * f);
                if (chg[u]) {
                    const u32 bc = (a.diag & 4) ? 0u : cc[u];
                    const float* bp = a.B + static_cast<size_t>(bc) * KT + W * sub;
#pragma unroll
                    for (int f = 0; f < NF; ++f)
                        bv[u][f] = *reinterpret_cast<const vt*>(bp + 16 * W * f);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (!chg[u]) {
#pragma unroll
                    for (int f = 0; f < NF; ++f) bv[u][f] = u ? bv[u - 1][f] : bcur[f];
                }
                float acc = 0.f;
#pragma unroll
                for (int f = 0; f < NF; ++f) acc += vdot<W>(av[u][f], bv[u][f]);
                acc = row_sum16(acc);
                // diag 1: store only an impossible value (keeps the math, drops the P scatter)
                if (sub == 0 && ok[u] && (!(a.diag & 1) || acc == -1234.5f)) a.P[oo[u]] = acc;
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (ok[u]) {
                    curc = cc[u];
#pragma unroll
                    for (int f = 0; f < NF; ++f) bcur[f] = bv[u][f];
                }
        }
    }
}

// ---- column-major residual slot, runtime K (multiple of 16): G = 4 lanes per entry
__device__ __forceinline__ void residual_cm_generic(const SddmmArgs& a, const uint2 sl) {
    constexpr u32 G = 4, NG = 16;
    const u32 l = __lane_id(), sub = l % G, grp = l / G;
    const u32 n = sl.y - sl.x;
    const u32 share = (n + NG - 1) / NG;
    const u32 gs = sl.x + min(grp * share, n), ge = sl.x + min(grp * share + share, n);
    for (u32 e = gs; e < ge; ++e) {
        const float* ap = a.A + static_cast<size_t>(a.cmRow[e]) * a.K;
        const float* bp = a.B + static_cast<size_t>(a.cmCol[e]) * a.K;
        float acc = 0.f;
        for (u32 k = 4 * sub; k < a.K; k += 4 * G) acc += dot4(ld4(ap + k), ld4(bp + k));
        acc = group_sum<G>(acc);
        if (sub == 0) a.P[a.cmOut[e]] = acc;
    }
}

// ---- panel-major residual item (panel ranges): A rows of the panel staged in LDS
template <int G>
__device__ __forceinline__ void residual_panel(const SddmmArgs& a, const uint4 it, float* As) {
    const u32 l = __lane_id();
    const u32 K = a.K, KP = K + 4;
    for (u32 x = 4 * l; x < 16 * K; x += 256) {
        const u32 r = x / K, k = x - r * K;
        const u32 q = it.x * 16 + r;
        const f32x4 v = q < a.R ? ld4(a.A + static_cast<size_t>(a.rows[q]) * K + k) : f32x4{0, 0, 0, 0};
        *reinterpret_cast<f32x4*>(As + r * KP + k) = v;
    }
    __syncthreads();
    constexpr u32 EPI = 64 / G;
    const u32 sub = l % G, grp = l / G;
    for (u32 base = it.y; base < it.z; base += EPI) {
        const u32 e = base + grp;
        const bool ok = e < it.z;
        const u32 ee = ok ? e : it.y;
        const float* brow = a.B + static_cast<size_t>(a.sparseCol[ee]) * K;
        const float* arow = As + a.sparseRel[ee] * KP;
        float acc = 0.f;
        for (u32 k = 4 * sub; k < K; k += 4 * G)
            acc += dot4(*reinterpret_cast<const f32x4*>(arow + k), ld4(brow + k));
        acc = group_sum<G>(acc);
        if (sub == 0 && ok) a.P[a.sparseValues[ee]] = acc;
    }
    __syncthreads();
}

// full launch: 256-thread workgroups of four independent waves, one work item per wave (no LDS,
// no barriers); <= 64 VGPRs so 8 waves per SIMD (32 per CU) are resident. Items [0, nd) are dense
// tiles, residual slots start at item ndpad = roundup(nd, 32), so slot s sits in block
// (ndpad + s) / 4 whose XCD (block % 8) is the slot's column bucket (slot layout in plan.hip).
template <int KT, int G>
__global__ __launch_bounds__(256, (KT >= 256 ? 4 : 8)) void k_sddmm_f32(SddmmArgs a) {
    const unsigned long long t0 = rtime(a.trace);
    if (blockIdx.y) {
        a.A += blockIdx.y * a.bA;
        a.B += blockIdx.y * a.bB;
        a.P += blockIdx.y * a.bP;
    }
    const u32 b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b < a.nd) {
        dense_tile<KT>(a, a.d0 + b);
        trace_wave(a.trace, b, t0, t0);
        return;
    }
    const u32 ndpad = (a.nd + 31) & ~31u;
    if (b < ndpad) return;
    const u32 s = b - ndpad;
    if (s < a.nslots) {
        const uint2 sl = a.slots[s];
        if (sl.x < sl.y) {
            if constexpr (KT > 0)
                residual_cm<KT>(a, sl);
            else
                residual_cm_generic(a, sl);
        }
    }
    trace_wave(a.trace, b, t0, t0);
}

// panel-range launch: dense items of the range, then its panel-major residual items
template <int KT, int G>
__global__ __launch_bounds__(64) void k_sddmm_panels_f32(SddmmArgs a) {
    extern __shared__ __attribute__((aligned(16))) float As[];
    const u32 b = blockIdx.x;
    if (b < a.nd) {
        dense_tile<KT>(a, a.d0 + b);
    } else if (b - a.nd < a.nr) {
        residual_panel<G>(a, a.ritems[a.r0 + b - a.nd], As);
    }
}

// ==========================================================================================
// Row-block launch (rows of RBY = 256 or 512 bytes: fp32 K = 64/128, fp16/bf16 K = 128/256): one
// workgroup per item {row block rb, tiles [t0, t1), residual pieces [p0, p1)} (layout:
// Plan::build_rowblock_layout). The A rows of the RB reordered positions of rb are staged in LDS
// once (<= 144 KiB); dense tiles take their MFMA A operand and residual entries their A pieces
// from LDS, so the only gathered operand is B, read once per column run (entries are sorted by
// (row block, column)).
//
// Residual entries: G = 4 lanes per entry (16 row-groups per wave), so the per-entry bookkeeping
// (metadata broadcast, addresses, store) is shared by 16 entries per wave instruction; each lane
// owns NC = RBY/64 16-byte chunks 4t + s of the row (packed FMA for fp32, v_dot2 for fp16/bf16,
// fp32 accumulation) and the quad reduces with two DPP adds.
// LDS image: row lr at lr * RBY bytes (unpadded); chunk c of row lr sits at
// (c & ~3) | ((c & 3) ^ (lr & 3)). Lane (row-group j, sub s) visits its chunks in the rotated
// order t = (f + j) mod NC, so in every ds_read_b128 lane group ({0-3,12-15,20-27},
// {4-11,16-19,28-31}, +32 = row-groups {0,3,5,6}, {1,2,4,7}, ...) the four row-groups read four
// different 64-byte quads: conflict-free for any rows (the XOR only permutes inside a quad).
// Dense tiles read chunk 16w + 4g + j of the 16 tile rows: the XOR spreads rows 0-3 (2-way).
// ==========================================================================================
struct RbArgs {
    const char* A;  // row-major M x K elements of the dtype
    const char* B;  // N rows of K elements (B column-major)
    float* P;
    const u32* rows;
    u32 R, N, RB;  // R: rows at or past this reordered position are not staged (range end)
    u32 qbase;     // reordered position of row block 0 (16 * first panel of the range)
    u32 row0;      // row staged for positions outside the block (its unused image tail): a row
                   // the launch's A holds (0, or 16 * first panel for a shard-local A)
    const uint4* items;     // {row block, tile begin, tile end, piece begin}
    const u32* itemEnd;     // piece end
    const uint2* pieces;    // {first entry, column | (length - 1) << 22}
    const u32* meta;        // local row << 22 | column
    const u32* out;
    const uint4* tilePanel;  // dense work items: .x = panel of the tile
    const u32* tileIds;      // the layout's kept tiles: item tile ranges index this list
    const u32* denseCols;
    const u32* blockValues;
    u32 mode;  // 1 = dense tiles, 2 = residual, 3 = both
    // staged output (Plan::RowBlockLayout::outLds): != 0 = byte offset of the item's result slots
    // in LDS; the entry metadata's low bits are then the slot, and the workgroup writes the slots
    // to P[sortedPos[itemEnt.x + t]] at the end
    u32 outLds;
    u32 outPacked;  // 1: no out array, the metadata's low 22 bits are the CSR position
    u32 stageNt;  // 1: stage the A rows with the nt policy (Plan::stage_nt)
    u32 lateB;    // 1: phase-0 B columns / metadata loaded after the staging barrier (late_b)
    u32 stageBlocks;  // 1 KiB LDS-DMA blocks that hold the image (RB * RBY / 1024); the rest of
                      // the workgroup's LDS is not staged
    const u32* sortedPos;
    const uint2* itemEnt;
    // staged output by runs (RowBlockLayout::outRuns; else null): {position, slot | len << 16}, len <= 64
    // per run of consecutive CSR positions, {first run, runs} per item
    const uint2* runs;
    const uint2* itemRuns;
    u32 pairs;  // 1: each workgroup runs list positions 2j and 2j + 1 of its XCD (see k_sddmm_rb)
    unsigned long long* trace;  // BSMR_DIAG & 32 timeline (see trace_wave)
    u32 diag;                   // profiling ablations (BSMR_DIAG); always 0 in normal use
    unsigned long long bA, bB, bP;  // batched launch: A, B byte strides, P element stride
};

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 b16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 b16x8 __attribute__((ext_vector_type(8)));

// physical 16-byte chunk of logical chunk c of image row lr. fp16/bf16 images swizzle inside each
// 64-byte quad so the MFMA tile reads (4 chunk-consecutive rows per lane group) spread over the
// banks; fp32 images are plain (no tiles on the fp32 row-block path; the residual reads are
// conflict-free by the rotation alone), which saves the swizzle arithmetic per entry.
template <int DT>
__device__ __forceinline__ u32 lds_chunk(u32 lr, u32 c) {
    if constexpr (DT == 0)
        return c;
    else
        return (c & ~3u) | ((c & 3u) ^ (lr & 3u));
}

__device__ __forceinline__ f32x4 ld16(const char* p) { return *reinterpret_cast<const f32x4*>(p); }

// one staging LDS-DMA wave-instruction: 16 bytes per lane from g to LDS at l + 16 * lane (l
// wave-uniform). Inline asm, so the compiler's wait-count pass does not track it: around the
// builtin, a branch (skipping the blocks past the image) made the compiler wait (vmcnt(0)) for
// every LDS-DMA before issuing the next. The kernels order these by their explicit
// s_waitcnt vmcnt(0) + barrier before the image is read. AUX 2: the nt cache policy.
// LDS byte address of a pointer into the workgroup's LDS
__device__ __forceinline__ u32 lds_addr(const char* l) {
    return __builtin_amdgcn_readfirstlane(static_cast<u32>(
        reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const char*)l)));
}
template <int AUX>
__device__ __forceinline__ void rb_dma16(const char* g, const u32 m0) {
    if constexpr (AUX == 2)
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off nt" ::"v"(g), "s"(m0)
                     : "memory", "m0");
    else
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m0)
                     : "memory", "m0");
}

// value of lane I of the quad in every lane of the quad
template <int I>
__device__ __forceinline__ u32 quad_bcast(u32 v) {
    return static_cast<u32>(
        __builtin_amdgcn_update_dpp(0, static_cast<int>(v), I * 0x55, 0xF, 0xF, false));
}

// acc += a . b over one 16-byte chunk (DT 0: 4 fp32, packed FMA; 1: 8 fp16, 2: 8 bf16, v_dot2)
template <int DT>
__device__ __forceinline__ void chunk_dot(const f32x4 a, const f32x4 b, f32x2& acc0, f32x2& acc1) {
    if constexpr (DT == 0) {
        acc0 = __builtin_elementwise_fma(f32x2{a.x, a.y}, f32x2{b.x, b.y}, acc0);
        acc1 = __builtin_elementwise_fma(f32x2{a.z, a.w}, f32x2{b.z, b.w}, acc1);
    } else if constexpr (DT == 1) {
        // whole-vector bit casts + swizzles: __builtin_bit_cast of a vector ELEMENT miscompiles
        // here (hipcc 7.2 reads element 0 for every index)
        const h16x8 ha = __builtin_bit_cast(h16x8, a), hb = __builtin_bit_cast(h16x8, b);
        acc0.x = __builtin_amdgcn_fdot2(ha.s01, hb.s01, acc0.x, false);
        acc0.y = __builtin_amdgcn_fdot2(ha.s23, hb.s23, acc0.y, false);
        acc1.x = __builtin_amdgcn_fdot2(ha.s45, hb.s45, acc1.x, false);
        acc1.y = __builtin_amdgcn_fdot2(ha.s67, hb.s67, acc1.y, false);
    } else {
        const b16x8 ha = __builtin_bit_cast(b16x8, a), hb = __builtin_bit_cast(b16x8, b);
        acc0.x = __builtin_amdgcn_fdot2_f32_bf16(ha.s01, hb.s01, acc0.x, false);
        acc0.y = __builtin_amdgcn_fdot2_f32_bf16(ha.s23, hb.s23, acc0.y, false);
        acc1.x = __builtin_amdgcn_fdot2_f32_bf16(ha.s45, hb.s45, acc1.x, false);
        acc1.y = __builtin_amdgcn_fdot2_f32_bf16(ha.s67, hb.s67, acc1.y, false);
    }
}

// acc += the MFMA of one 16-byte A chunk and B chunk per lane (DT 0: four 16x16x4 f32 steps;
// 1/2: one 16x16x32 f16/bf16 step), lane layout of dense_tile (one k-block per lane group)
template <int DT>
__device__ __forceinline__ f32x4 chunk_mfma(const f32x4 a, const f32x4 b, f32x4 acc) {
    if constexpr (DT == 0) {
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc, 0, 0, 0);
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc, 0, 0, 0);
    } else if constexpr (DT == 1) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h16x8, a),
                                                      __builtin_bit_cast(h16x8, b), acc, 0, 0, 0);
    } else {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b16x8, a),
                                                       __builtin_bit_cast(b16x8, b), acc, 0, 0, 0);
    }
}

// lanes per residual entry for a row size: 4 up to 512-byte rows, 8 for 1 KiB, 16 for 2 KiB rows;
// every lane then owns NC = RBY / (16 * G) <= 8 chunks of the row
template <int RBY>
struct RowGeom {
    static constexpr u32 G = RBY >= 2048 ? 16 : RBY >= 1024 ? 8 : 4;
    static constexpr u32 NC = RBY / (16 * G);
    static constexpr u32 NB = (RB_PIECE_MAX + G - 1) / G;  // metadata batches per piece
    // distinct chunk-group rotations the residual reads need: a ds_read_b128 lane group
    // (MI355X_MICROARCH.md §LDS: {0-3,12-15,20-27}, {4-11,16-19,28-31}, +32) holds 4 row-groups
    // of 4 lanes whose 64-byte reads must fill the 256-byte bank row (rotations j mod 4 differ
    // inside each), halves of 4 8-lane groups (j mod 2 moves them by 128 bytes), or one 16-lane
    // group that already spans it. Reads f <= NC - RR never wrap, so they address one base
    // register with immediate offsets.
    static constexpr u32 RR = (G == 4 ? 4u : G == 8 ? 2u : 1u) < NC ? (G == 4 ? 4u : G == 8 ? 2u : 1u) : NC;
};

// value of lane I of the G-lane group in every lane of the group
template <int G, int I>
__device__ __forceinline__ u32 group_bcast(u32 v) {
    if constexpr (G == 4)
        return quad_bcast<I>(v);
    else if constexpr (G == 8)  // ds_swizzle bit mode: and 0x18 (the group), or I
        return static_cast<u32>(__builtin_amdgcn_ds_swizzle(static_cast<int>(v), 0x18 | (I << 5)));
    else  // a whole DPP row
        return row_bcast<I>(v);
}

// dense tile on the LDS image: load() gathers the tile's metadata and B operand (no LDS, so a
// wave can issue it before the staging barrier), run() reads the A rows from LDS, runs the MFMAs
// and scatters the 256 outputs. Lane group g takes chunk 16w + 4g + j at k-step 4w + j (any
// k-permutation shared by A and B is valid), so the XOR of the LDS image spreads it. Rows of
// 1 KiB (16 chunks per lane) are processed in two halves of 8 chunks.
template <int DT, int RBY>
struct DenseTileLds {
    static constexpr int NK = RBY / 64;          // 16-byte chunks per lane
    static constexpr int CH = NK > 8 ? 8 : NK;   // chunks held in registers at once
    u32 lr, c, idx[4];
    __device__ __forceinline__ static u32 chunk(int kk, u32 g) {
        if constexpr (NK >= 4)
            return 16 * (kk >> 2) + 4 * g + (kk & 3);
        else  // 128-byte rows: k-step kk covers chunks kk, NK + kk, 2 NK + kk, 3 NK + kk
            return NK * g + kk;
    }
    __device__ __forceinline__ void meta(const RbArgs& a, const u32 tile, const u32 q0) {
        const u32 l = __lane_id(), rr = l & 15, g = l >> 4;
        const u32 p = a.tilePanel[tile].x;
        c = a.denseCols[tile * 16 + rr];
        const u32* bvals = a.blockValues + static_cast<size_t>(tile) * 256 + 64 * g + rr;
#pragma unroll
        for (int r = 0; r < 4; ++r) idx[r] = bvals[16 * r];
        lr = p * 16 - q0 + rr;
    }
    // B chunks [k0, k0 + CH)
    __device__ __forceinline__ void loadB(const RbArgs& a, const int k0, f32x4 (&bv)[CH]) const {
        const u32 g = __lane_id() >> 4;
        const bool cvalid = c < a.N;
        // BSMR_DIAG & 8388608 (ablation only): every tile reads B column 0, so its gathers hit L2
        const char* bcol = a.B + static_cast<size_t>(cvalid && !(a.diag & 8388608u) ? c : 0) * RBY;
#pragma unroll
        for (int kk = 0; kk < CH; ++kk)
            bv[kk] = cvalid ? ld16(bcol + 16 * chunk(k0 + kk, g)) : f32x4{0, 0, 0, 0};
    }
    __device__ __forceinline__ void load(const RbArgs& a, const u32 tile, const u32 q0,
                                         f32x4 (&bv)[CH]) {
        meta(a, tile, q0);
        loadB(a, 0, bv);
    }
    // bv: the first CH chunks (from load); later halves are loaded here
    __device__ __forceinline__ void run(const RbArgs& a, const char* As, f32x4 (&bv)[CH]) const {
        const u32 g = __lane_id() >> 4;
        const char* arow = As + lr * RBY;
        f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
#pragma unroll
        for (int k0 = 0; k0 < NK; k0 += CH) {
            if (k0) loadB(a, k0, bv);
#pragma unroll
            for (int kk = 0; kk < CH; ++kk) {
                const f32x4 av = ld16(arow + 16 * lds_chunk<DT>(lr, chunk(k0 + kk, g)));
                f32x4& acc = (kk & 1) ? acc1 : acc0;
                acc = chunk_mfma<DT>(av, bv[kk], acc);
            }
        }
        const f32x4 acc = acc0 + acc1;
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (idx[r] != NULLV) a.P[idx[r]] = acc[r];
    }
};

// B pieces of the group's column (lane s: chunks G * ((f + j) mod NC) + s, f < NC)
template <int RBY>
__device__ __forceinline__ void load_bcol(const RbArgs& a, const u32 col, const u32 sub,
                                          const u32 (&rot)[RowGeom<RBY>::NC],
                                          f32x4 (&bv)[RowGeom<RBY>::NC]) {
    // B < 4 GiB on this path (rb_slot); BSMR_DIAG & 64 (ablation only): every piece reads
    // column 0, so the B gathers hit L2
    const u32 bb = ((a.diag & 64) ? 0u : col) * RBY + 16 * sub;
#pragma unroll
    for (u32 f = 0; f < RowGeom<RBY>::NC; ++f)
        bv[f] = f + RowGeom<RBY>::RR <= RowGeom<RBY>::NC
                    ? ld16(a.B + (bb + rot[0]) + 16 * RowGeom<RBY>::G * f)  // no wrap: immediate
                    : ld16(a.B + (bb + rot[f]));
}

// a column-run piece of a row-group: entries [first, first + len), len <= RB_PIECE_MAX, all
// in one column. Lane s of the group holds the metadata of entries first + G*k + s.
template <int RBY>
struct Piece {
    u32 first, len, col;
    u32 mm[RowGeom<RBY>::NB], mo[RowGeom<RBY>::NB];
};

// the piece descriptor (first entry, column, length)
template <int RBY>
__device__ __forceinline__ void load_piece_desc(const RbArgs& a, const u32 pi, Piece<RBY>& pc) {
    const uint2 d = a.pieces[pi];
    pc.first = d.x;
    pc.len = (d.y >> 22) + 1;
    pc.col = d.y & 0x3FFFFFu;
}

// the piece's B column and its entries' metadata (after load_piece_desc)
template <int RBY>
__device__ __forceinline__ void load_piece_body(const RbArgs& a, const u32 sub,
                                                const u32 (&rot)[RowGeom<RBY>::NC],
                                                f32x4 (&bv)[RowGeom<RBY>::NC], Piece<RBY>& pc) {
    constexpr u32 G = RowGeom<RBY>::G;
    load_bcol<RBY>(a, pc.col, sub, rot, bv);
#pragma unroll
    for (u32 k = 0; k < RowGeom<RBY>::NB; ++k) {
        const u32 e = G * k + sub;
        pc.mm[k] = e < pc.len ? a.meta[pc.first + e] : 0u;
        // staged output: the slot is the metadata's low bits, taken where the result is stored
        // (deriving it here made the prologue wait for this load, and so for the B column
        // before it, ahead of the staging)
        pc.mo[k] = !a.outLds && !a.outPacked && e < pc.len ? a.out[pc.first + e] : 0u;
    }
}

template <int RBY>
__device__ __forceinline__ void load_piece(const RbArgs& a, const u32 pi, const u32 sub,
                                           const u32 (&rot)[RowGeom<RBY>::NC],
                                           f32x4 (&bv)[RowGeom<RBY>::NC], Piece<RBY>& pc) {
    load_piece_desc<RBY>(a, pi, pc);
    load_piece_body<RBY>(a, sub, rot, bv, pc);
}

// Step i of a batch of G computes entry G*k + i in all G lanes; lane i keeps it, so a batch ends
// in one store instruction for G entries per group (64 outputs per full wave).
template <int DT, int RBY>
__device__ __forceinline__ void residual_piece(const RbArgs& a, const char* As,
                                               const Piece<RBY>& pc, const u32 sub,
                                               const u32 (&rot)[RowGeom<RBY>::NC],
                                               const f32x4 (&bv)[RowGeom<RBY>::NC]) {
    constexpr u32 G = RowGeom<RBY>::G, NC = RowGeom<RBY>::NC;
#pragma unroll
    for (u32 k = 0; k < RowGeom<RBY>::NB; ++k) {
        if (G * k >= pc.len) break;
        const u32 nb = min(G, pc.len - G * k);
        // fp32 images are unswizzled: broadcast the image row offset lr * RBY itself, computed
        // once per batch by the lane that owns the entry, instead of shifting m in every step
        const u32 mk = DT == 0 ? (pc.mm[k] >> 22) * RBY : pc.mm[k];
        float res = 0.f;
#pragma unroll
        for (int i = 0; i < static_cast<int>(G); ++i) {
            if (static_cast<u32>(i) >= nb) break;
            u32 m;
            switch (i) {
#define BSMR_C(I) \
    case I: m = group_bcast<G, (I < G ? I : 0)>(mk); break;
                BSMR_C(0) BSMR_C(1) BSMR_C(2) BSMR_C(3) BSMR_C(4) BSMR_C(5) BSMR_C(6) BSMR_C(7)
                BSMR_C(8) BSMR_C(9) BSMR_C(10) BSMR_C(11) BSMR_C(12) BSMR_C(13) BSMR_C(14)
#undef BSMR_C
                default: m = group_bcast<G, G - 1>(mk); break;
            }
            u32 ab;  // + rot[f]: chunk G t + sub
            if constexpr (DT == 0) {
                ab = m + 16 * sub;
            } else {
                const u32 lr = m >> 22;
                ab = lr * RBY + 16 * lds_chunk<DT>(lr, sub);
            }
            const char* arot = As + (ab + rot[0]);                   // no wrap before f = NC - RR
            f32x2 acc0 = {0.f, 0.f}, acc1 = {0.f, 0.f};
            constexpr u32 H = NC > 4 ? NC / 2 : NC;  // LDS reads in flight per half
#pragma unroll
            for (u32 h = 0; h < NC; h += H) {
                f32x4 av[H];
#pragma unroll
                for (u32 f = 0; f < H; ++f)
                    av[f] = h + f + RowGeom<RBY>::RR <= NC ? ld16(arot + 16 * G * (h + f))
                                                           : ld16(As + (ab + rot[h + f]));
#pragma unroll
                for (u32 f = 0; f < H; ++f) {
                    if constexpr (DT == 0)  // one packed chain: no acc0 + acc1 per entry
                        chunk_dot<DT>(av[f], bv[h + f], acc0, acc0);
                    else
                        chunk_dot<DT>(av[f], bv[h + f], acc0, acc1);
                }
            }
            f32x2 acc = acc0;
            if constexpr (DT != 0) acc += acc1;
            float sm = acc.x + acc.y;
            sm += dppf<0xB1>(sm);                         // quad_perm [1,0,3,2]
            sm += dppf<0x4E>(sm);                         // quad_perm [2,3,0,1]
            if constexpr (G >= 8) sm += dppf<0x141>(sm);   // row_half_mirror: the other quad
            if constexpr (G == 16) sm += dppf<0x140>(sm);  // row_mirror: the other half-row
            if (sub == static_cast<u32>(i)) res = sm;
        }
        if (sub < nb) {
            if (a.outLds)  // the slot: rank by CSR position inside the item
                *reinterpret_cast<float*>(const_cast<char*>(As) + a.outLds +
                                          4 * (pc.mm[k] & 0x3FFFFFu)) = res;
            else
                a.P[a.outPacked ? pc.mm[k] & 0x3FFFFFu : pc.mo[k]] = res;
        }
    }
}

// Dynamic piece batches (RowBlockLayout::dynBatches, rows of <= 512 B): batch b = the item's
// pieces [b GW, (b + 1) GW), GW = 64 / G, one per row-group of a wave. Wave w runs batch w first
// (the static phase 0), then takes the next batch from a counter in the workgroup's last LDS word
// (the layout keeps it free), so waves whose pieces were short or whose gathers were fast take
// more of an item with many pieces per row-group. The next batch's piece is loaded while the
// current one computes, as in the static phases. Returns after the wave's last batch.
constexpr u32 BATCH_CTR_BYTES = 16;  // the counter's share of the workgroup's LDS (its end)
template <int DT, int RBY, int NT, typename LoadRuns>
__device__ __forceinline__ void rb_batches(const RbArgs& a, const char* As, const u32 p0, const u32 np,
                                           const u32 gr, const u32 sub, const u32 (&rot)[RowGeom<RBY>::NC],
                                           Piece<RBY>& pc, f32x4 (&pre)[RowGeom<RBY>::NC], LoadRuns&& load_runs) {
    constexpr u32 NC = RowGeom<RBY>::NC, GW = 64 / RowGeom<RBY>::G, NW = NT / 64;
    u32* const ctr = reinterpret_cast<u32*>(const_cast<char*>(As) + (NT == 1024 ? 160u : 80u) * 1024u - 4u);
    auto grab = [&]() -> u32 {
        u32 v = 0;
        if ((threadIdx.x & 63) == 0)
            v = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return NW + static_cast<u32>(__builtin_amdgcn_readfirstlane(static_cast<int>(v)));
    };
    Piece<RBY> pn;
    f32x4 nb[NC];
    auto fetch = [&](const u32 b) {
        const u32 pi = b * GW + gr % GW;
        pn.len = 0;
        if (pi < np) load_piece<RBY>(a, p0 + pi, sub, rot, nb, pn);
    };
    u32 bn = grab();
    if (bn * GW < np)
        fetch(bn);
    else
        load_runs();
    if (pc.len) residual_piece<DT, RBY>(a, As, pc, sub, rot, pre);
    while (bn * GW < np) {
        pc = pn;
#pragma unroll
        for (u32 f = 0; f < NC; ++f) pre[f] = nb[f];
        bn = grab();
        if (bn * GW < np)
            fetch(bn);
        else
            load_runs();
        if (pc.len) residual_piece<DT, RBY>(a, As, pc, sub, rot, pre);
    }
}

constexpr u32 NO_ITEM = 0xFFFFFFFFu;
// run values a wave holds in registers while the next item's staging is issued (pairs)
constexpr u32 PAIR_RUNS_PER_WAVE = 16;

// staging row indices of the row block starting at reordered position q0, one per lane (rows of
// >= 256 bytes: lane l holds the row of block w + (l / NR) NW, rows l % NR of it)
template <int RBY, int NT>
__device__ __forceinline__ u32 rb_stage_rows(const RbArgs& a, const u32 q0, const u32 ws, const u32 lane) {
    constexpr u32 NW = NT / 64, NCH = RBY / 16, NR = NCH >= 64 ? 1 : 64 / NCH;
    constexpr u32 MAXB = (NT == 1024 ? 160u : 80u) / NW;
    const u32 i = lane / NR, b = ws + i * NW, lr = 64 * b / NCH + lane % NR, q = q0 + lr;
    return (i < MAXB && lr < a.RB && q < a.R) ? a.rows[q] : a.row0;
}

// the LDS-DMAs of one row block (rows of >= 256 bytes; rowv from rb_stage_rows): every wave
// issues its 1 KiB blocks of the image back to back (see k_sddmm_rb)
template <int DT, int RBY, int NT, int AUX>
__device__ __forceinline__ void rb_stage_issue(const RbArgs& a, char* As, u32 rowv, const u32 ws,
                                               const u32 lane) {
    constexpr u32 NW = NT / 64, NCH = RBY / 16, NR = NCH >= 64 ? 1 : 64 / NCH;
    // the row indices in registers before the first LDS-DMA: the compiler does not count the
    // (inline asm) DMAs, so a wait for the indices inside the rolled loop (at its head) would also
    // wait for every DMA issued before it
    asm volatile("" : "+v"(rowv));
    constexpr u32 MAXB = (NT == 1024 ? 160u : 80u) / NW;
    const u32 x0 = 64 * ws + lane;
    const u32 coff = 16 * lds_chunk<DT>(x0 / NCH, x0 % NCH);
    // (a loop rolled by two: fully unrolled, its v_readlane results were all hoisted into SGPRs,
    // which the pair kernel's two items cannot spare)
#pragma unroll 2
    for (u32 i = 0; i < MAXB; ++i) {
        const u32 b = ws + i * NW;
        u32 src = static_cast<u32>(__builtin_amdgcn_readlane(static_cast<int>(rowv), i * NR));
#pragma unroll
        for (u32 k = 1; k < NR; ++k) {
            const u32 rk = static_cast<u32>(__builtin_amdgcn_readlane(static_cast<int>(rowv), i * NR + k));
            src = lane / NCH == k ? rk : src;
        }
        const char* g = a.A + (static_cast<size_t>(src) * RBY + coff);
        if (b < a.stageBlocks) rb_dma16<AUX>(g, lds_addr(As) + 1024 * b);
    }
}

// One row-block work item (see k_sddmm_rb). prestaged: the previous item of the workgroup's pair
// already issued this item's staging. next (pairs, staged output by runs): the item that runs
// next on this workgroup; its staging is issued in this item's store pass, right after the result
// slots have been read into registers, so the next image lands while this item's stores drain.
// Returns whether next's staging was issued (false: next is padding, or this item holds more
// runs per wave than PAIR_RUNS_PER_WAVE and stored them the plain way).
template <int DT, int RBY, int NT, int OM, bool DYN = false>
__device__ __forceinline__ bool rb_item(const RbArgs& a, char* As, const u32 idx, const bool prestaged,
                                        const u32 next) {
    // OM (output mode): 0 = one store per entry (a.outLds == 0), 1 = staged output (slots in
    // LDS, written per item in CSR order), 2 = staged output by runs in pairs (PAIR; LEAN: no
    // kept tiles, trace or ablations)
    constexpr bool PAIR = OM == 2, STAGED = OM != 0, LEAN = OM >= 2;
    using Geo = RowGeom<RBY>;
    constexpr u32 G = Geo::G, NC = Geo::NC;  // lanes per entry, chunks per lane
    constexpr u32 NW = NT / 64;               // waves per workgroup
    constexpr u32 NG = NT / G;                // residual row-groups
    constexpr u32 TC = DenseTileLds<DT, RBY>::CH;
    // the pair kernel (PAIR): staged output by runs, no kept MFMA tiles, late B loads, default
    // staging policy, no trace or ablations (launch_rb picks it only then): its two items fit
    // the SGPR budget without those paths
    const unsigned long long t0 = LEAN ? 0ull : rtime(a.trace);
    uint4 it = a.items[idx];
    // all four fields in SGPRs before the padding test: the compiler otherwise loads .x (the row
    // block) in a second, dependent round trip after the test
    it.x = __builtin_amdgcn_readfirstlane(it.x);
    it.y = __builtin_amdgcn_readfirstlane(it.y);
    it.z = __builtin_amdgcn_readfirstlane(it.z);
    it.w = __builtin_amdgcn_readfirstlane(it.w);
    const u32 pend = a.itemEnd[idx];
    if (it.y == it.z && it.w == pend) return false;  // padding item (uniform across the workgroup)
    // the next item of the pair: its row block (its staging rows are loaded in the last phase)
    bool has_next = false, same_rb = false;
    u32 q0n = 0;
    if (next != NO_ITEM) {
        uint4 nt = a.items[next];
        nt.x = __builtin_amdgcn_readfirstlane(nt.x);
        nt.y = __builtin_amdgcn_readfirstlane(nt.y);
        nt.z = __builtin_amdgcn_readfirstlane(nt.z);
        nt.w = __builtin_amdgcn_readfirstlane(nt.w);
        const u32 nend = __builtin_amdgcn_readfirstlane(a.itemEnd[next]);
        has_next = !(nt.y == nt.z && nt.w == nend);
        q0n = a.qbase + nt.x * a.RB;
        // the same row block (consecutive chunks of one segment): its image is already in LDS
        // (the pieces only read it; the slots live past it), so nothing is staged again
        same_rb = nt.x == it.x;
    }
    const u32 q0 = a.qbase + it.x * a.RB;
    u32 tid = threadIdx.x;
    // LEAN (two items per workgroup): the thread-derived values are recomputed per item
    // rather than hoisted out of the caller's loop, where they would hold VGPRs across it
    if constexpr (LEAN) asm volatile("" : "+v"(tid));
    const u32 w = tid >> 6, sub = tid % G, j = (tid & 63) / G;
    // every wave takes (at most) one dense tile and its row-groups one residual piece each per
    // phase; the first tile and the phase-0 pieces (B operand, metadata) are issued before the
    // staging loads so all of it is in flight together
    const u32 ntile = !LEAN && (a.mode & 1) ? it.z - it.y : 0u;
    const u32 np = (a.mode & 2) ? pend - it.w : 0u;
    const u32 gr = tid / G;
    u32 rot[NC];  // residual: byte offset of the G-chunk group the lane visits at step f
#pragma unroll
    for (u32 f = 0; f < NC; ++f) rot[f] = 16u * G * ((f + j % Geo::RR) % NC);
    // stage the row block by LDS-DMA: each wave-instruction fills one contiguous KiB of the image
    // (64 chunks of the row-major image); lane l supplies image chunk x = 64 b + l, i.e. row
    // lr = x / NCH at physical chunk pc = x % NCH, read from the logical chunk lds_chunk(lr, pc)
    // of A[rows[q0 + lr]] (the XOR is an involution). The row indices of the wave's blocks are
    // loaded once, one per lane, and handed to the block's lanes with v_readlane + select.
    // Wave w stages the image's blocks b = w + i NW < stageBlocks, back to back, by inline-asm
    // LDS-DMAs (rb_dma16): around the builtin, a branch (skipping a block) or any LDS instruction
    // between two LDS-DMAs made the compiler wait (vmcnt(0)) for each LDS-DMA before issuing the
    // next, which serialised the staging (C2: 12.8 -> 12.0 us once removed); until round 5 every
    // wave therefore staged the launch's whole LDS, the blocks past the image reading row 0.
    constexpr u32 NCH = RBY / 16;
    constexpr u32 NR = NCH >= 64 ? 1 : 64 / NCH;  // rows a block starts (<= 4)
    constexpr u32 MAXB = (NT == 1024 ? 160u : 80u) / NW;
    static_assert(MAXB * NW == (NT == 1024 ? 160u : 80u), "whole KiB blocks");
    constexpr bool ROWV = MAXB * NR <= 64;  // one row index per lane (else 128-byte rows)
    const u32 lane = tid & 63;
    const u32 ws = __builtin_amdgcn_readfirstlane(w);  // wave index in an SGPR
    // the staging row indices are loaded first: they depend only on the item, so their round
    // trip overlaps the piece descriptor's, and the LDS-DMAs need not wait for the B columns
    u32 rowv = 0;  // (set before every staging: rb_stage_rows, or the pair's next rows)
    u32 src[ROWV ? 1 : MAXB];
    if (!prestaged) {
        if constexpr (ROWV) {
            rowv = rb_stage_rows<RBY, NT>(a, q0, ws, lane);
        } else {
            // 128-byte rows: 8 rows per block, too many indices for one per lane; each lane
            // loads the row of its own chunk for every block
#pragma unroll
            for (u32 i = 0; i < MAXB; ++i) {
                const u32 lr = 64 * (ws + i * NW) / NCH + lane / NCH, q = q0 + lr;
                src[i] = lr < a.RB && q < a.R ? a.rows[q] : a.row0;
            }
            // all row indices in registers before the first LDS-DMA: the compiler does not count
            // the (inline asm) DMAs, so a wait for a later index placed between them would also
            // wait for the DMAs issued before it (mycielskian14 K = 32: 16.3 -> 17.7 us)
#pragma unroll
            for (u32 i = 0; i < MAXB; ++i) asm volatile("" : "+v"(src[i]));
        }
    }
    // the loads the LDS-DMA issue waits for go first: row indices, the phase-0 piece descriptor
    // and the first tile's metadata (one round trip together); the B columns and entry metadata
    // they address are issued after the LDS-DMAs, so the staging never waits for a B gather
    f32x4 tb[TC], pre[NC];
    DenseTileLds<DT, RBY> dt;
    // tiles go to the last waves, which hold the shortest pieces (pieces are sorted longest first)
    const u32 tw = NW - 1 - w;
    Piece<RBY> pc;
    pc.len = 0;
    if constexpr (!LEAN)
        if (tw < ntile) dt.meta(a, a.tileIds[it.y + tw], q0);
    if (gr < np) load_piece_desc<RBY>(a, it.w + gr, pc);
    // staged output by runs: this lane's run descriptor (run w + NW * lane of the item), loaded
    // when the wave's pieces are done, so the store pass waits (at most) for the slowest wave's
    // descriptors; with a next item, its staging row indices are loaded there too
    uint2 myrun = make_uint2(0u, 0u), irun = make_uint2(0u, 0u);
    u32 rown = a.row0;
    auto load_runs = [&]() {
        if (STAGED && a.runs && a.outLds) {
            irun = a.itemRuns[idx];
            irun.x = __builtin_amdgcn_readfirstlane(irun.x);
            irun.y = __builtin_amdgcn_readfirstlane(irun.y);
            const u32 jr = w + NW * lane;
            if (jr < irun.y) myrun = a.runs[irun.x + jr];
        }
        if constexpr (ROWV)
            if (has_next && !same_rb) rown = rb_stage_rows<RBY, NT>(a, q0n, ws, lane);
    };
    // AUX: the LDS-DMA cache policy (0 default; 2 = nt, stream the A rows past the XCD's L2 so the
    // B columns of the item's column range stay resident: large staged-output layouts, where an
    // item's row block is not staged again on that XCD until the next range)
    auto stage = [&](auto aux_tag) {
        constexpr int AUX = decltype(aux_tag)::value;
        if constexpr (ROWV) {
            rb_stage_issue<DT, RBY, NT, AUX>(a, As, rowv, ws, lane);
        } else {
            // the source chunk of lane l is the same in every block of the wave: x % NCH and
            // (x / NCH) & 3 for x = 64 (ws + i NW) + l do not depend on i (NW = 16 or 8, NCH >= 8)
            const u32 x0 = 64 * ws + lane;
            const u32 coff = 16 * lds_chunk<DT>(x0 / NCH, x0 % NCH);
#pragma unroll
            for (u32 i = 0; i < MAXB; ++i) {
                const u32 b = ws + i * NW;
                const char* g = a.A + (static_cast<size_t>(src[i]) * RBY + coff);
                if (b < a.stageBlocks) rb_dma16<AUX>(g, lds_addr(As) + 1024 * b);
            }
        }
    };
    if (!prestaged) {
        if (!LEAN && a.stageNt)  // (LEAN: the launch takes the default policy)
            stage(std::integral_constant<int, 2>{});
        else
            stage(std::integral_constant<int, 0>{});
    }
    // the phase-0 B columns and entry metadata: issued right behind the LDS-DMAs (so the
    // barrier's wait covers them too), or with lateB after the barrier (the barrier then waits
    // for the staging alone and the waves pay one load round trip before their first piece)
    if (!LEAN && !a.lateB) {
        if (gr < np) load_piece_body<RBY>(a, sub, rot, pre, pc);
        if (tw < ntile) dt.loadB(a, 0, tb);
    }
    // every LDS-DMA of the workgroup has landed before any wave reads the image or writes the
    // staged-output slots (the blocks past the image land in the tail those slots use); explicit,
    // not left to the compiler's wait insertion at the barrier
    // the batch counter (no LDS-DMA writes the last word; every grab of the pair's previous item
    // ended before its store-pass barrier)
    if constexpr (DYN)
        if (tid == 0) *reinterpret_cast<u32*>(As + (NT == 1024 ? 160u : 80u) * 1024u - 4u) = 0u;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (LEAN || a.lateB) {
        if (gr < np) load_piece_body<RBY>(a, sub, rot, pre, pc);
        if constexpr (!LEAN)
            if (tw < ntile) dt.loadB(a, 0, tb);
    }
    const unsigned long long tm = LEAN ? 0ull : rtime(a.trace);
    if (!LEAN && (a.diag & 8)) {  // staging only
        trace_wave(a.trace, idx * NW + w, t0, tm);
        return false;
    }
    if constexpr (!LEAN)
        if (tw < ntile) dt.run(a, As, tb);
    const unsigned long long td = LEAN ? 0ull : rtime(a.trace);
    // later phases (items with more pieces than row-groups, e.g. short column runs): phase ph
    // runs the column window [ph NG, (ph + 1) NG) of the item's pieces (longest first inside;
    // Plan::build_rowblock_layout), dealt forwards in even and backwards in odd phases so a wave
    // alternates long and short pieces; phase ph's piece and B column are loaded while phase
    // ph - 1 computes (two register sets)
    if constexpr (DYN) {
        rb_batches<DT, RBY, NT>(a, As, it.w, np, gr, sub, rot, pc, pre, [] {});
    } else {
        Piece<RBY> pn;
        f32x4 nb[NC];
        auto fetch = [&](const u32 ph) {
            const u32 pi = ph * NG + ((ph & 1) ? NG - 1 - gr : gr);
            pn.len = 0;
            if (pi < np) load_piece<RBY>(a, it.w + pi, sub, rot, nb, pn);
        };
        if (NG < np) fetch(1);
        if (pc.len) residual_piece<DT, RBY>(a, As, pc, sub, rot, pre);
        for (u32 ph = 1; ph * NG < np; ++ph) {
            pc = pn;
#pragma unroll
            for (u32 f = 0; f < NC; ++f) pre[f] = nb[f];
            if ((ph + 1) * NG < np) fetch(ph + 1);
            if (pc.len) residual_piece<DT, RBY>(a, As, pc, sub, rot, pre);
        }
    }
    // (behind the pieces, not in their last phase: live across the phase loop, the descriptors
    // cost the loop VGPRs; a wave that ends early has them back before the store-pass barrier)
    if constexpr (STAGED) load_runs();
    if constexpr (!LEAN) {
        for (u32 t = it.y + tw + NW; t < it.z; t += NW) {  // tiles beyond one per wave
            dt.load(a, a.tileIds[t], q0, tb);
            dt.run(a, As, tb);
        }
    }
    bool staged_next = false;
    if (STAGED && a.outLds) {  // the item's results in CSR order: runs of consecutive positions
        __syncthreads();
        const uint2 ie = a.itemEnt[idx];
        const float* res = reinterpret_cast<const float*>(As + a.outLds);
        const u32 nr = irun.y > w ? (irun.y - w + NW - 1) / NW : 0u;
        if constexpr (PAIR && ROWV) {
            // pairs: this wave's run values into registers, a barrier (no wave reads a slot
            // any more; the next image may reach into the slots), the next item's LDS-DMAs,
            // then this item's stores, all in flight together
            if (has_next && __builtin_amdgcn_readfirstlane(irun.y) <= NW * PAIR_RUNS_PER_WAVE) {
                float v[PAIR_RUNS_PER_WAVE];
#pragma unroll
                for (u32 u = 0; u < PAIR_RUNS_PER_WAVE; ++u) {
                    const u32 sl = static_cast<u32>(__builtin_amdgcn_readlane(static_cast<int>(myrun.y), u));
                    const u32 len = u < nr ? sl >> 16 : 0u;
                    v[u] = lane < len ? res[(sl & 0xFFFFu) + lane] : 0.0f;
                }
                __syncthreads();
                rowv = rown;
                if (!same_rb) stage(std::integral_constant<int, 0>{});
#pragma unroll
                for (u32 u = 0; u < PAIR_RUNS_PER_WAVE; ++u) {
                    const u32 pos = static_cast<u32>(__builtin_amdgcn_readlane(static_cast<int>(myrun.x), u));
                    const u32 sl = static_cast<u32>(__builtin_amdgcn_readlane(static_cast<int>(myrun.y), u));
                    const u32 len = u < nr ? sl >> 16 : 0u;
                    if (lane < len) a.P[pos + lane] = v[u];
                }
                return true;
            }
        }
        if (LEAN || !(a.diag & 128)) {  // (BSMR_DIAG & 128, ablation only: no P stores)
            if (LEAN || a.runs) {
                // wave w writes runs w, w + NW, ...: one contiguous store of up to 64 results
                // per run (a row's results in this item, when rows are column-sorted), four
                // runs per step with their LDS reads in flight together
                for (u32 i = 0; i < nr; i += 4) {
                    u32 pos[4], s0[4], len[4];
                    float v[4];
#pragma unroll
                    for (u32 u = 0; u < 4; ++u) {
                        const u32 q = min(i + u, 63u);
                        pos[u] = static_cast<u32>(__builtin_amdgcn_readlane(static_cast<int>(myrun.x), q));
                        const u32 sl = static_cast<u32>(__builtin_amdgcn_readlane(static_cast<int>(myrun.y), q));
                        s0[u] = sl & 0xFFFFu;
                        len[u] = i + u < nr ? sl >> 16 : 0u;
                        v[u] = lane < len[u] ? res[s0[u] + lane] : 0.0f;
                    }
#pragma unroll
                    for (u32 u = 0; u < 4; ++u)  // (runs are at most 64 long)
                        if (lane < len[u]) a.P[pos[u] + lane] = v[u];
                }
            } else if constexpr (!LEAN) {
                // eight position loads in flight per lane before their stores: a loop of
                // dependent load -> store pairs exposed one L2 latency per 1024 results (C4 x0.5:
                // 1.135 -> 1.082 ms). Issuing the first batch before the barrier measured slower
                constexpr u32 U = 8;
                for (u32 t0s = tid; t0s < ie.y; t0s += U * NT) {
                    u32 pos[U];
#pragma unroll
                    for (u32 k = 0; k < U; ++k) {
                        const u32 t = t0s + k * NT;
                        pos[k] = t < ie.y ? a.sortedPos[ie.x + t] : 0u;
                    }
#pragma unroll
                    for (u32 k = 0; k < U; ++k) {
                        const u32 t = t0s + k * NT;
                        if (t < ie.y) a.P[pos[k]] = res[t];
                    }
                }
            }
        }
        // a pair whose first item stored the plain way: the next image is staged now (every
        // slot read has completed at the barrier)
        if constexpr (PAIR && ROWV) {
            if (has_next) {
                __syncthreads();
                rowv = rown;
                if (!same_rb) stage(std::integral_constant<int, 0>{});
                staged_next = true;
            }
        }
    }
    if constexpr (!LEAN) trace_wave(a.trace, idx * NW + w, t0, tm, td);
    return staged_next;
}

// Row-block SDDMM: one workgroup per work item {row block, kept-tile range, piece
// range}: the row block's A rows staged in LDS, then its MFMA tiles and column-run pieces, then
// (staged output) the item's results in CSR order.
// (This single-item kernel keeps its own body rather than calling rb_item: the shared form
// measured 3 % slower on C2, 10.70 vs 10.46 us on one box, with the same instruction count; the
// pair kernel below uses rb_item.)
// LITE: the form the C2-like launches take — no kept MFMA tiles, one store per entry (no staged
// output), default staging policy, phase-0 B after the barrier, no trace or ablations (launch_rb
// picks it only then): the same instructions on that path, without the code of the others
template <int DT, int RBY, int NT, bool DYN, bool LITE = false>
__global__ __launch_bounds__(NT, 4) void k_sddmm_rb(RbArgs a) {
    extern __shared__ __attribute__((aligned(16))) char AsB[];
    char* As = AsB;
    if (blockIdx.y) {  // batch b (item -> XCD placement unchanged: nItems is a multiple of 8)
        a.A += blockIdx.y * a.bA;
        a.B += blockIdx.y * a.bB;
        a.P += blockIdx.y * a.bP;
    }
    using Geo = RowGeom<RBY>;
    constexpr u32 G = Geo::G, NC = Geo::NC;  // lanes per entry, chunks per lane
    constexpr u32 NW = NT / 64;               // waves per workgroup
    constexpr u32 NG = NT / G;                // residual row-groups
    constexpr u32 TC = DenseTileLds<DT, RBY>::CH;
    const unsigned long long t0 = LITE ? 0ull : rtime(a.trace);
    uint4 it = a.items[blockIdx.x];
    // all four fields in SGPRs before the padding test: the compiler otherwise loads .x (the row
    // block) in a second, dependent round trip after the test
    it.x = __builtin_amdgcn_readfirstlane(it.x);
    it.y = __builtin_amdgcn_readfirstlane(it.y);
    it.z = __builtin_amdgcn_readfirstlane(it.z);
    it.w = __builtin_amdgcn_readfirstlane(it.w);
    const u32 pend = a.itemEnd[blockIdx.x];
    if (it.y == it.z && it.w == pend) return;  // padding item (uniform across the workgroup)
    const u32 q0 = a.qbase + it.x * a.RB;
    const u32 tid = threadIdx.x, w = tid >> 6, sub = tid % G, j = (tid & 63) / G;
    // every wave takes (at most) one dense tile and its row-groups one residual piece each per
    // phase; the first tile and the phase-0 pieces (B operand, metadata) are issued before the
    // staging loads so all of it is in flight together
    const u32 ntile = !LITE && (a.mode & 1) ? it.z - it.y : 0u;
    const u32 np = LITE || (a.mode & 2) ? pend - it.w : 0u;
    const u32 gr = tid / G;
    u32 rot[NC];  // residual: byte offset of the G-chunk group the lane visits at step f
#pragma unroll
    for (u32 f = 0; f < NC; ++f) rot[f] = 16u * G * ((f + j % Geo::RR) % NC);
    // stage the row block by LDS-DMA: each wave-instruction fills one contiguous KiB of the image
    // (64 chunks of the row-major image); lane l supplies image chunk x = 64 b + l, i.e. row
    // lr = x / NCH at physical chunk pc = x % NCH, read from the logical chunk lds_chunk(lr, pc)
    // of A[rows[q0 + lr]] (the XOR is an involution). The row indices of the wave's blocks are
    // loaded once, one per lane, and handed to the block's lanes with v_readlane + select.
    // Wave w stages the image's blocks b = w + i NW < stageBlocks, back to back, by inline-asm
    // LDS-DMAs (rb_dma16): around the builtin, a branch (skipping a block) or any LDS instruction
    // between two LDS-DMAs made the compiler wait (vmcnt(0)) for each LDS-DMA before issuing the
    // next, which serialised the staging (C2: 12.8 -> 12.0 us once removed); until round 5 every
    // wave therefore staged the launch's whole LDS, the blocks past the image reading row 0.
    constexpr u32 NCH = RBY / 16;
    constexpr u32 NR = NCH >= 64 ? 1 : 64 / NCH;  // rows a block starts (<= 4)
    constexpr u32 MAXB = (NT == 1024 ? 160u : 80u) / NW;
    static_assert(MAXB * NW == (NT == 1024 ? 160u : 80u), "whole KiB blocks");
    constexpr bool ROWV = MAXB * NR <= 64;  // one row index per lane (else 128-byte rows)
    const u32 lane = tid & 63;
    const u32 ws = __builtin_amdgcn_readfirstlane(w);  // wave index in an SGPR
    // the staging row indices are loaded first: they depend only on the item, so their round
    // trip overlaps the piece descriptor's, and the LDS-DMAs need not wait for the B columns
    u32 rowv = a.row0;
    u32 src[ROWV ? 1 : MAXB];
    if constexpr (ROWV) {
        const u32 i = lane / NR, b = ws + i * NW, lr = 64 * b / NCH + lane % NR, q = q0 + lr;
        if (i < MAXB && lr < a.RB && q < a.R) rowv = a.rows[q];
    } else {
        // 128-byte rows: 8 rows per block, too many indices for one per lane; each lane loads
        // the row of its own chunk for every block
#pragma unroll
        for (u32 i = 0; i < MAXB; ++i) {
            const u32 lr = 64 * (ws + i * NW) / NCH + lane / NCH, q = q0 + lr;
            src[i] = lr < a.RB && q < a.R ? a.rows[q] : a.row0;
        }
        // all row indices in registers before the first LDS-DMA: the compiler does not count
        // the (inline asm) DMAs, so a wait for a later index placed between them would also
        // wait for the DMAs issued before it (mycielskian14 K = 32: 16.3 -> 17.7 us)
#pragma unroll
        for (u32 i = 0; i < MAXB; ++i) asm volatile("" : "+v"(src[i]));
    }
    // the loads the LDS-DMA issue waits for go first: row indices, the phase-0 piece descriptor
    // and the first tile's metadata (one round trip together); the B columns and entry metadata
    // they address are issued after the LDS-DMAs, so the staging never waits for a B gather
    f32x4 tb[TC], pre[NC];
    DenseTileLds<DT, RBY> dt;
    // tiles go to the last waves, which hold the shortest pieces (pieces are sorted longest first)
    const u32 tw = NW - 1 - w;
    Piece<RBY> pc;
    pc.len = 0;
    if constexpr (!LITE)
        if (tw < ntile) dt.meta(a, a.tileIds[it.y + tw], q0);
    if (gr < np) load_piece_desc<RBY>(a, it.w + gr, pc);
    // staged output by runs: this lane's run descriptor (run w + NW * lane of the item), loaded
    // in the item's last piece phase, where the next-phase prefetch registers are free, so the
    // store pass waits for nothing but the LDS slots
    uint2 myrun = make_uint2(0u, 0u), irun = make_uint2(0u, 0u);
    auto load_runs = [&]() {
        if (!LITE && a.runs && a.outLds) {
            irun = a.itemRuns[blockIdx.x];
            irun.x = __builtin_amdgcn_readfirstlane(irun.x);
            irun.y = __builtin_amdgcn_readfirstlane(irun.y);
            const u32 j = w + NW * lane;
            if (j < irun.y) myrun = a.runs[irun.x + j];
        }
    };
    // AUX: the LDS-DMA cache policy (0 default; 2 = nt, stream the A rows past the XCD's L2 so the
    // B columns of the item's column range stay resident: large staged-output layouts, where an
    // item's row block is not staged again on that XCD until the next range)
    auto stage = [&](auto aux_tag) {
        constexpr int AUX = decltype(aux_tag)::value;
        // the source chunk of lane l is the same in every block of the wave: x % NCH and
        // (x / NCH) & 3 for x = 64 (ws + i NW) + l do not depend on i (NW = 16 or 8, NCH >= 8)
        const u32 x0 = 64 * ws + lane;
        const u32 coff = 16 * lds_chunk<DT>(x0 / NCH, x0 % NCH);
        if constexpr (ROWV) {
#pragma unroll
            for (u32 i = 0; i < MAXB; ++i) {
                const u32 b = ws + i * NW;
                u32 src = static_cast<u32>(__builtin_amdgcn_readlane(static_cast<int>(rowv), i * NR));
#pragma unroll
                for (u32 k = 1; k < NR; ++k) {
                    const u32 rk = static_cast<u32>(__builtin_amdgcn_readlane(static_cast<int>(rowv), i * NR + k));
                    src = lane / NCH == k ? rk : src;
                }
                const char* g = a.A + (static_cast<size_t>(src) * RBY + coff);
                if (b < a.stageBlocks) rb_dma16<AUX>(g, lds_addr(As) + 1024 * b);
            }
        } else {
#pragma unroll
            for (u32 i = 0; i < MAXB; ++i) {
                const u32 b = ws + i * NW;
                const char* g = a.A + (static_cast<size_t>(src[i]) * RBY + coff);
                if (b < a.stageBlocks) rb_dma16<AUX>(g, lds_addr(As) + 1024 * b);
            }
        }
    };
    if (!LITE && a.stageNt)
        stage(std::integral_constant<int, 2>{});
    else
        stage(std::integral_constant<int, 0>{});
    // the phase-0 B columns and entry metadata: issued right behind the LDS-DMAs (so the
    // barrier's wait covers them too), or with lateB after the barrier (the barrier then waits
    // for the staging alone and the waves pay one load round trip before their first piece)
    if (!LITE && !a.lateB) {
        if (gr < np) load_piece_body<RBY>(a, sub, rot, pre, pc);
        if (tw < ntile) dt.loadB(a, 0, tb);
    }
    // every LDS-DMA of the workgroup has landed before any wave reads the image or writes the
    // staged-output slots (the blocks past the image land in the tail those slots use); explicit,
    // not left to the compiler's wait insertion at the barrier
    if constexpr (DYN)  // (the image-only staging never writes the last word)
        if (tid == 0) *reinterpret_cast<u32*>(As + (NT == 1024 ? 160u : 80u) * 1024u - 4u) = 0u;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (LITE || a.lateB) {
        if (gr < np) load_piece_body<RBY>(a, sub, rot, pre, pc);
        if constexpr (!LITE)
            if (tw < ntile) dt.loadB(a, 0, tb);
    }
    const unsigned long long tm = LITE ? 0ull : rtime(a.trace);
    if (!LITE && (a.diag & 8)) {  // staging only
        trace_wave(a.trace, blockIdx.x * NW + w, t0, tm);
        return;
    }
    if constexpr (!LITE)
        if (tw < ntile) dt.run(a, As, tb);
    const unsigned long long td = LITE ? 0ull : rtime(a.trace);
    // later phases (items with more pieces than row-groups, e.g. short column runs): phase ph
    // runs the column window [ph NG, (ph + 1) NG) of the item's pieces (longest first inside;
    // Plan::build_rowblock_layout), dealt forwards in even and backwards in odd phases so a wave
    // alternates long and short pieces; phase ph's piece and B column are loaded while phase
    // ph - 1 computes (two register sets)
    if constexpr (DYN) {
        rb_batches<DT, RBY, NT>(a, As, it.w, np, gr, sub, rot, pc, pre, load_runs);
    } else {
        Piece<RBY> pn;
        f32x4 nb[NC];
        auto fetch = [&](const u32 ph) {
            const u32 pi = ph * NG + ((ph & 1) ? NG - 1 - gr : gr);
            pn.len = 0;
            if (pi < np) load_piece<RBY>(a, it.w + pi, sub, rot, nb, pn);
        };
        if (NG < np)
            fetch(1);
        else
            load_runs();
        if (pc.len) residual_piece<DT, RBY>(a, As, pc, sub, rot, pre);
        for (u32 ph = 1; ph * NG < np; ++ph) {
            pc = pn;
#pragma unroll
            for (u32 f = 0; f < NC; ++f) pre[f] = nb[f];
            if ((ph + 1) * NG < np)
                fetch(ph + 1);
            else
                load_runs();
            if (pc.len) residual_piece<DT, RBY>(a, As, pc, sub, rot, pre);
        }
    }
    if constexpr (LITE) return;
    for (u32 t = it.y + tw + NW; t < it.z; t += NW) {  // tiles beyond one per wave
        dt.load(a, a.tileIds[t], q0, tb);
        dt.run(a, As, tb);
    }
    if (a.outLds) {  // the item's results in CSR order: runs of consecutive positions
        __syncthreads();
        const uint2 ie = a.itemEnt[blockIdx.x];
        const float* res = reinterpret_cast<const float*>(As + a.outLds);
        if (!(a.diag & 128)) {  // (BSMR_DIAG & 128, ablation only: no P stores)
            // eight position loads in flight per lane before their stores: a loop of dependent
            // load -> store pairs exposed one L2 latency per 1024 results (C4 x0.5: 1.135 ->
            // 1.082 ms). Issuing the first batch before the barrier measured slower (1.109 ms)
            constexpr u32 U = 8;
            auto pass = [&]() {
                for (u32 t0 = tid; t0 < ie.y; t0 += U * NT) {
                    u32 pos[U];
#pragma unroll
                    for (u32 k = 0; k < U; ++k) {
                        const u32 t = t0 + k * NT;
                        pos[k] = t < ie.y ? a.sortedPos[ie.x + t] : 0u;
                    }
#pragma unroll
                    for (u32 k = 0; k < U; ++k) {
                        const u32 t = t0 + k * NT;
                        if (t < ie.y) a.P[pos[k]] = res[t];
                    }
                }
            };
            if (a.runs) {
                // wave w writes runs w, w + NW, ...: one contiguous store of up to 64 results
                // per run (a row's results in this item, when rows are column-sorted), four
                // runs per step with their LDS reads in flight together
                const u32 nr = irun.y > w ? (irun.y - w + NW - 1) / NW : 0u;
                for (u32 i = 0; i < nr; i += 4) {
                    u32 pos[4], s0[4], len[4];
                    float v[4];
#pragma unroll
                    for (u32 u = 0; u < 4; ++u) {
                        const u32 q = min(i + u, 63u);
                        pos[u] = static_cast<u32>(__builtin_amdgcn_readlane(static_cast<int>(myrun.x), q));
                        const u32 sl = static_cast<u32>(__builtin_amdgcn_readlane(static_cast<int>(myrun.y), q));
                        s0[u] = sl & 0xFFFFu;
                        len[u] = i + u < nr ? sl >> 16 : 0u;
                        v[u] = lane < len[u] ? res[s0[u] + lane] : 0.0f;
                    }
#pragma unroll
                    for (u32 u = 0; u < 4; ++u)  // (runs are at most 64 long)
                        if (lane < len[u]) a.P[pos[u] + lane] = v[u];
                }
            } else {
                pass();
            }
        }
    }
    trace_wave(a.trace, blockIdx.x * NW + w, t0, tm, td);
}

// Pairs (staged output by runs): a workgroup runs list positions 2j and 2j + 1 of its XCD
// (items are laid out [position * 8 + x]; workgroup g runs on XCD g % 8), the second item's
// staging issued in the first one's store pass (rb_item)
template <int DT, int RBY, int NT, bool DYN>
__global__ __launch_bounds__(NT, 4) void k_sddmm_rb_pair(RbArgs a) {
    extern __shared__ __attribute__((aligned(16))) char AsB[];
    char* As = AsB;
    if (blockIdx.y) {  // batch b
        a.A += blockIdx.y * a.bA;
        a.B += blockIdx.y * a.bB;
        a.P += blockIdx.y * a.bP;
    }
    const u32 x = blockIdx.x % XCD_BUCKETS, i0 = (blockIdx.x / XCD_BUCKETS) * 2 * XCD_BUCKETS + x;
    if (rb_item<DT, RBY, NT, 2, DYN>(a, As, i0, false, i0 + XCD_BUCKETS))
        rb_item<DT, RBY, NT, 2, DYN>(a, As, i0 + XCD_BUCKETS, true, NO_ITEM);
}

template <int DT, int RBY>
void (*pick_rb(const u32 NT, const bool pairs, const bool dyn, const bool lite))(RbArgs) {
    // (dynamic batches: rows of <= 512 B, RowBlockLayout::dynBatches)
    if constexpr (RBY >= 256) {  // (launch_rb enables pairs from 512-byte rows)
        if (pairs) {
            if constexpr (RBY <= 512)
                if (dyn) return NT == 1024 ? k_sddmm_rb_pair<DT, RBY, 1024, true> : k_sddmm_rb_pair<DT, RBY, 512, true>;
            return NT == 1024 ? k_sddmm_rb_pair<DT, RBY, 1024, false> : k_sddmm_rb_pair<DT, RBY, 512, false>;
        }
    }
    if constexpr (RBY <= 512)
        if (dyn) {
            if (lite) return NT == 1024 ? k_sddmm_rb<DT, RBY, 1024, true, true> : k_sddmm_rb<DT, RBY, 512, true, true>;
            return NT == 1024 ? k_sddmm_rb<DT, RBY, 1024, true> : k_sddmm_rb<DT, RBY, 512, true>;
        }
    if (lite) return NT == 1024 ? k_sddmm_rb<DT, RBY, 1024, false, true> : k_sddmm_rb<DT, RBY, 512, false, true>;
    return NT == 1024 ? k_sddmm_rb<DT, RBY, 1024, false> : k_sddmm_rb<DT, RBY, 512, false>;
}

static_assert(TILES_PER_ITEM == 1, "dense work items are single tiles (tile id = item id)");

using KernelFn = void (*)(SddmmArgs);

template <int G, bool PANELS>
KernelFn pick_k(u32 K) {
#define BSMR_K(KT) (PANELS ? k_sddmm_panels_f32<KT, G> : k_sddmm_f32<KT, G>)
    switch (K) {
        case 32: return BSMR_K(32);
        case 64: return BSMR_K(64);
        case 128: return BSMR_K(128);
        case 256: return BSMR_K(256);
        case 512: return BSMR_K(512);
        default: return BSMR_K(0);
    }
#undef BSMR_K
}

template <bool PANELS>
KernelFn pick_kernel(u32 K) {
    if (K % 64 == 0) return pick_k<16, PANELS>(K);
    if (K % 32 == 0) return pick_k<8, PANELS>(K);
    return pick_k<4, PANELS>(K);
}

int validate(const void* dA, const void* dB, u32 K, int dtype, const float* dP) {
    if (!dA || !dB || !dP) {
        set_error("bsmr_sddmm: null device pointer");
        return BSMR_ERR_INVALID;
    }
    if (K == 0 || K % 16 != 0) {
        set_error("bsmr_sddmm: K must be a positive multiple of 16");
        return BSMR_ERR_UNSUPPORTED;
    }
    if (dtype != BSMR_F32 && dtype != BSMR_F16 && dtype != BSMR_BF16) {
        set_error("bsmr_sddmm: dtype must be BSMR_F32, BSMR_F16 or BSMR_BF16");
        return BSMR_ERR_UNSUPPORTED;
    }
    return BSMR_OK;
}

SddmmArgs make_args(const Plan& p, const void* dA, const void* dB, u32 K, float* dP) {
    SddmmArgs a{};
    a.A = static_cast<const float*>(dA);
    a.B = static_cast<const float*>(dB);
    a.P = dP;
    a.tileRows = p.tileRows.data();
    a.rows = p.rows.data();
    a.R = p.R;
    a.N = p.N;
    a.K = K;
    a.denseCols = p.denseCols.data();
    a.blockValues = p.blockValues.data();
    a.slots = p.cmSlots.data();
    a.cmRow = p.cmRow.data();
    a.cmCol = p.cmCol.data();
    a.cmOut = p.cmOut.data();
    a.ritems = p.resItems.data();
    a.sparseValues = p.sparseValues.data();
    a.sparseRel = p.sparseRel.data();
    a.sparseCol = p.sparseColIdx.data();
    a.diag = p.diag;
    return a;
}

// (K, dtype) -> row-block layout slot by row bytes (0..3: 256 B .. 2 KiB); -1: the column-major
// path
int rb_slot(const Plan& p, u32 K, int dtype) {
    if (p.N > (1u << 22) || !p.use_rowblock) return -1;
    // tile-dominated plans (e.g. 16x16 block masks): one tile per wave with A from L2 beats
    // staging row blocks (C5 block mask: 8.9 vs 11.1 us); row blocks pay off once the residual
    // carries a quarter of the work (a tile ~ 16 entries)
    if (!p.force_rowblock && static_cast<u64>(p.nres) * 4 < static_cast<u64>(p.numDenseTiles) * 16)
        return -1;
    const u32 rby = K * (dtype == BSMR_F32 ? 4u : 2u);
    // the row-block kernel addresses B with 32-bit byte offsets (load_bcol): B < 4 GiB
    if (static_cast<u64>(p.N) * rby >= (1ull << 32)) return -1;
    return rby == 128 ? 0 : rby == 256 ? 1 : rby == 512 ? 2 : rby == 1024 ? 3 : rby == 2048 ? 4 : -1;
}

// fp16/bf16 patterns dense enough for whole MFMA tiles (sddmm_dense.hip)
bool use_dense(const Plan& p, u32 K, int dtype) {
    // layout auto only (BSMR_LAYOUT_ROWBLOCK / _COLMAJOR force those launches); bsmr_sddmm asks
    // use_ptile first (tile-dominated fp16/bf16 plans, K in {64..512}: C5 block 7.8 -> 5.6 us)
    // tile-dominated plans (16 x 16 block masks) keep the column-major tile launch below K = 512:
    // a 128 x 128 tile's fixed prologue and epilogue only pay off over long K (C5 block mask,
    // bf16: dense 8.2 vs 8.9 us at K = 512, 5.95 vs 5.35 at 256, 4.7 vs 3.8 at 128;
    // profiles/r02c/dense_blockmask_ab.txt)
    if (K < 512 && static_cast<u64>(p.nres) * 4 < static_cast<u64>(p.numDenseTiles) * 16) return false;
    return p.use_rowblock && !p.force_rowblock && dtype != BSMR_F32 && K % 64 == 0 &&
           static_cast<double>(p.nnz) >= static_cast<double>(p.dense_min) * p.M * static_cast<double>(p.N);
}

// tile-dominated fp16/bf16 plans (16 x 16 block masks: residual under a quarter of the work) with
// K in {64, 128, 256, 512}: the panel-grouped tile launch (sddmm_half.hip k_sddmm_ptile), every
// BSMR tile on MFMA with the panel's A rows staged once per item (BSMR_PTILE = 1: whenever the
// dtype and K allow, also beside a large residual; 0: never)
bool use_ptile(const Plan& p, u32 K, int dtype) {
    if (dtype == BSMR_F32 || p.ptile_mode == 0 || !p.use_rowblock || p.force_rowblock) return false;
    if ((K != 64 && K != 128 && K != 256 && K != 512) || p.numDenseTiles == 0) return false;
    return p.ptile_mode == 1 ||
           static_cast<u64>(p.nres) * 4 < static_cast<u64>(p.numDenseTiles) * 16;
}

// the row-block layout of panels [pa, pb) for slot's row size (built on first use)
int get_rb_layout(const Plan& p, int slot, int dtype, u32 pa, u32 pb,
                  std::shared_ptr<const Plan::RowBlockLayout>* out) {
    std::lock_guard<std::mutex> g(p.layout_mu);
    int err = BSMR_OK;
    *out = p.rowblock_layout(128u << slot, dtype != BSMR_F32, pa, pb, &err);
    return err;
}

// mode: 1 = dense tiles only, 2 = residual only, 3 = both (profiling splits). local: dA holds
// the rows of reordered positions [16 L.pa, L.rowEnd) in that order (row-panel shard with its
// own A rows): the launch stages them through the identity row list, from dA shifted back by
// 16 L.pa rows (addresses only; no row before 16 L.pa is read)
int launch_rb(const Plan& p, const Plan::RowBlockLayout& L, const void* dA, const void* dB,
              float* dP, int dtype, u32 mode, hipStream_t s, u32 nb = 1, bool local = false) {
    if (L.nItems == 0) return BSMR_OK;
    RbArgs a{};
    a.A = static_cast<const char*>(dA);
    if (local)
        a.A = reinterpret_cast<const char*>(reinterpret_cast<uintptr_t>(dA) -
                                            static_cast<uintptr_t>(16ull * L.pa * L.rowBytes));
    a.B = static_cast<const char*>(dB);
    // column blocks: B's rows are the staged image, A's the gathered rows (the kernel computes
    // the same dot products with the operands' roles swapped)
    if (L.cols) std::swap(a.A, a.B);
    a.P = dP;
    a.rows = local ? p.iotaR.data() : (L.orig || L.cols) ? L.rowIds.data() : p.rows.data();
    a.row0 = local ? 16 * L.pa : 0;
    a.R = L.rowEnd;
    a.qbase = (L.orig || L.cols) ? 0 : 16 * L.pa;
    a.N = L.cols ? p.M : p.N;
    a.RB = L.RB;
    a.items = L.items.data();
    a.itemEnd = L.itemEnd.data();
    a.pieces = L.pieces.data();
    a.meta = L.meta.data();
    a.out = L.out.data();
    a.outLds = (mode & 2) ? L.outLds : 0u;  // (dense-only profiling launches write no slots)
    a.outPacked = L.outPacked ? 1u : 0u;
    a.stageNt = p.stage_nt == 1 || (p.stage_nt == -1 && L.outLds != 0 && p.stage_nt_auto);
    a.lateB = p.late_b != 0;
    // the image's blocks only (BSMR_DIAG & 2097152, A/B only: every block of the launch's LDS but
    // the last, which holds the piece-batch counter — the filler past the image reading row 0, as
    // before round 5)
    a.stageBlocks = (p.diag & 2097152u) ? (L.NT == 1024 ? 159u : 79u)
                                        : (L.RB * L.rowBytes + 1023) / 1024;
    a.sortedPos = L.sortedPos.data();
    a.itemEnt = L.itemEnt.data();
    a.runs = L.outRuns ? L.runs.data() : nullptr;
    a.itemRuns = L.outRuns ? L.itemRuns.data() : nullptr;
    // pairs (BSMR_DIAG & 16384 off): staged output by runs, rows of >= 512 bytes, at least 4096
    // items (16 rounds of the chip's workgroup slots), an even number of list positions per XCD;
    // not under the profiling ablations (trace, staging only, B in L2, no stores). A pair is two
    // items long, so short lists lose to the tail: mycielskian15 K = 64 / 128 (832 / 728 items)
    // 56.9 / 74.6 us paired against 50.1 / 66.5 unpaired, mycielskian16 K = 64 114.6 against
    // 108.9; C4 (8-30 K items) gains (x0.5 1.029 -> 0.984 ms), C3, mycielskian16 K = 128 and
    // 1-2 KiB rows are neutral (profiles/r04zt, r04zw)
    a.pairs = mode == 3 && rb_uses_pairs(p, L) ? 1u : 0u;
    a.tilePanel = p.denseItems.data();
    a.tileIds = L.tileIds.data();
    a.denseCols = p.denseCols.data();
    a.blockValues = p.blockValues.data();
    a.mode = mode;
    a.diag = p.diag;
    if (p.diag & 32) {
        BSMR_CHECK(p.prepare_trace(static_cast<size_t>(L.nItems) * (L.NT / 64), s));
        a.trace = p.trace.data();
    }
    a.bA = static_cast<unsigned long long>(L.cols ? p.N : p.M) * L.rowBytes;
    a.bB = static_cast<unsigned long long>(L.cols ? p.M : p.N) * L.rowBytes;
    a.bP = p.nnz;
    void (*fn)(RbArgs) = nullptr;
    // the LITE single-item kernel: the whole launch (mode 3), no kept tiles, direct stores, default
    // staging policy, late B, no trace or ablation bits (BSMR_DIAG & 33554432 keeps the full form
    // for A/B)
    const bool lite = mode == 3 && L.nTilesKept == 0 && !a.outLds && !a.stageNt && a.lateB && p.diag == 0;
#define BSMR_RB(DT, RBY) pick_rb<DT, RBY>(L.NT, a.pairs != 0, L.dynBatches, lite)
#define BSMR_RB2(DT)                                                                   \
    (L.rowBytes == 128    ? BSMR_RB(DT, 128)                                              \
     : L.rowBytes == 256  ? BSMR_RB(DT, 256)                                              \
     : L.rowBytes == 512  ? BSMR_RB(DT, 512)                                              \
     : L.rowBytes == 1024 ? BSMR_RB(DT, 1024)                                             \
                          : BSMR_RB(DT, 2048))
    switch (dtype) {
        case BSMR_F32: fn = BSMR_RB2(0); break;
        case BSMR_F16: fn = BSMR_RB2(1); break;
        default: fn = BSMR_RB2(2); break;
    }
#undef BSMR_RB2
#undef BSMR_RB
    // the workgroup's LDS: 160 / 80 KiB (the image, the staged-output slots, the batch counter)
    const u32 grid = a.pairs ? L.nItems / 2 : L.nItems;
    hipLaunchKernelGGL(fn, dim3(grid, nb), dim3(L.NT),
                       (L.NT == 1024 ? 160 : 80) * 1024, s, a);
    BSMR_HIP(hipGetLastError());
    return BSMR_OK;
}

int launch_full(const Plan& p, SddmmArgs a, hipStream_t s, u32 nb = 1) {
    const u32 items = a.nslots ? ((a.nd + 31) & ~31u) + a.nslots : a.nd;
    if (items == 0) return BSMR_OK;
    a.bA = static_cast<unsigned long long>(p.M) * a.K;
    a.bB = static_cast<unsigned long long>(p.N) * a.K;
    a.bP = p.nnz;
    if (p.diag & 32) {
        BSMR_CHECK(p.prepare_trace((items + 3) / 4 * 4, s));
        a.trace = p.trace.data();
    }
    hipLaunchKernelGGL(pick_kernel<false>(a.K), dim3((items + 3) / 4, nb), dim3(256), 0, s, a);
    BSMR_HIP(hipGetLastError());
    return BSMR_OK;
}

int launch_panels(SddmmArgs a, hipStream_t s) {
    const u32 grid = a.nd + a.nr;
    if (grid == 0) return BSMR_OK;
    const size_t lds = a.nr ? static_cast<size_t>(16) * (a.K + 4) * sizeof(float) : 0;
    hipLaunchKernelGGL(pick_kernel<true>(a.K), dim3(grid), dim3(64), lds, s, a);
    BSMR_HIP(hipGetLastError());
    return BSMR_OK;
}

}  // namespace

// pairs (BSMR_DIAG & 16384 off): staged output by runs, rows of >= 512 bytes, at least
// pair_min_items (4096: 16 rounds of the chip's workgroup slots) items, an even number of list
// positions per XCD, no kept MFMA tile; not under the profiling ablations (trace, staging only, B
// in L2, no stores) nor nt staging / early B loads
bool rb_uses_pairs(const Plan& p, const Plan::RowBlockLayout& L) {
    const bool stageNt = p.stage_nt == 1 || (p.stage_nt == -1 && L.outLds != 0 && p.stage_nt_auto);
    return L.outRuns && L.outLds && L.rowBytes >= 512 && L.nItems >= p.pair_min_items &&
           L.nTilesKept == 0 && L.nItems % (2 * XCD_BUCKETS) == 0 && !stageNt && p.late_b != 0 &&
           !(p.diag & (8u | 32u | 64u | 128u | 16384u));
}

// whether bsmr_sddmm runs the dense-sampled launch for (K, dtype) (plan_check.cpp)
bool sddmm_uses_dense(const Plan& p, u32 K, int dtype) { return use_dense(p, K, dtype); }
// whether bsmr_sddmm runs the panel-grouped tile launch for (K, dtype) (plan_check.cpp, stats)
bool sddmm_uses_ptile(const Plan& p, u32 K, int dtype) { return use_ptile(p, K, dtype); }

// the whole plan's row-block layout for (K, dtype), built on first use; *out = null when that
// (K, dtype) runs the column-major launch
int whole_rb_layout(const Plan& p, u32 K, int dtype, const Plan::RowBlockLayout** out,
                    bool reordered) {
    *out = nullptr;
    const int slot = rb_slot(p, K, dtype);
    if (slot < 0 || use_ptile(p, K, dtype)) return BSMR_OK;
    std::shared_ptr<const Plan::RowBlockLayout> L;  // the whole plan's: a plan member
    BSMR_CHECK(get_rb_layout(p, slot, dtype, 0, p.P, &L));
    *out = L.get();
    // reordered: the reordered-row layout (always built first; panel shards cut its row blocks)
    if (reordered && (L->orig || L->cols)) *out = &p.rbl[slot + (dtype != BSMR_F32 ? Plan::N_RB_SIZES : 0)];
    return BSMR_OK;
}

}  // namespace bsmr

using namespace bsmr;

// one launch per at most 65535 batches (grid.y); batch b reads A + b*M*K, B + b*N*K and writes
// P + b*nnz (sddmm_gpu_batch, sddmmKernel.cu:2764-2850)
extern "C" int bsmr_sddmm_batch(const bsmr_plan* plan, uint32_t num_batch, const void* dA,
                                const void* dB, uint32_t K, int dtype, float* dP, void* stream) {
    if (!plan) {
        set_error("bsmr_sddmm: null plan");
        return BSMR_ERR_INVALID;
    }
    if (num_batch == 0) {
        set_error("bsmr_sddmm_batch: num_batch must be >= 1");
        return BSMR_ERR_INVALID;
    }
    const Plan& p = plan->p;
    BSMR_CHECK(validate(dA, dB, K, dtype, dP));
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const size_t es = dtype == BSMR_F32 ? 4 : 2;
    for (u32 b0 = 0; b0 < num_batch; b0 += 65535u) {
        const u32 nb = std::min<u32>(num_batch - b0, 65535u);
        const char* A = static_cast<const char*>(dA) + es * b0 * static_cast<size_t>(p.M) * K;
        const char* B = static_cast<const char*>(dB) + es * b0 * static_cast<size_t>(p.N) * K;
        float* P = dP + static_cast<size_t>(b0) * p.nnz;
        if (use_ptile(p, K, dtype)) {
            BSMR_CHECK(launch_ptile(p, A, B, K, dtype, P, 3, s, nb));
            continue;
        }
        if (use_dense(p, K, dtype)) {
            BSMR_CHECK(launch_dense(p, A, B, K, dtype, P, s, nb));
            continue;
        }
        const int slot = rb_slot(p, K, dtype);
        if (slot >= 0) {
            std::shared_ptr<const Plan::RowBlockLayout> L;
            BSMR_CHECK(get_rb_layout(p, slot, dtype, 0, p.P, &L));
            BSMR_CHECK(launch_rb(p, *L, A, B, P, dtype, 3, s, nb));
            continue;
        }
        if (dtype != BSMR_F32) {
            BSMR_CHECK(launch_half(p, A, B, K, dtype, P, 3, s, nb));
            continue;
        }
        SddmmArgs a = make_args(p, A, B, K, P);
        a.nd = p.nDenseItems;
        a.nslots = p.nSlots;
        BSMR_CHECK(launch_full(p, a, s, nb));
    }
    return BSMR_OK;
}

extern "C" int bsmr_sddmm(const bsmr_plan* plan, const void* dA, const void* dB, uint32_t K,
                          int dtype, float* dP, void* stream) {
    return bsmr_sddmm_batch(plan, 1, dA, dB, K, dtype, dP, stream);
}

extern "C" int bsmr_sddmm_panels(const bsmr_plan* plan, const void* dA, const void* dB,
                                 uint32_t K, int dtype, float* dP, uint32_t p0, uint32_t p1,
                                 void* stream) {
    if (!plan) {
        set_error("bsmr_sddmm_panels: null plan");
        return BSMR_ERR_INVALID;
    }
    const Plan& p = plan->p;
    BSMR_CHECK(validate(dA, dB, K, dtype, dP));
    if (p0 > p1 || p1 > p.P) {
        set_error("bsmr_sddmm_panels: bad panel range");
        return BSMR_ERR_INVALID;
    }
    if (p0 == p1) return BSMR_OK;
    // the row-block kernel over the range's own layout (same kernel as the whole plan)
    const int slot = rb_slot(p, K, dtype);
    if (slot >= 0) {
        std::shared_ptr<const Plan::RowBlockLayout> L;  // held until the launch is enqueued
        BSMR_CHECK(get_rb_layout(p, slot, dtype, p0, p1, &L));
        return launch_rb(p, *L, dA, dB, dP, dtype, 3, static_cast<hipStream_t>(stream));
    }
    if (dtype != BSMR_F32) {
        set_error("bsmr_sddmm_panels: fp16/bf16 panel ranges need the row-block layout "
                  "(half K in 128..1024)");
        return BSMR_ERR_UNSUPPORTED;
    }
    // items are stored panel-major: ceil(tiles_q / TILES_PER_ITEM) dense and
    // ceil(nres_q / RES_PER_ITEM) residual items per panel q
    u32 d0 = 0, d1 = 0, r0 = 0, r1 = 0;
    for (u32 q = 0; q < p1; ++q) {
        const u32 nt = p.h_blockOffsets[q + 1] - p.h_blockOffsets[q];
        const u32 ne = p.h_sparseValueOffsets[q + 1] - p.h_sparseValueOffsets[q];
        const u32 di = (nt + TILES_PER_ITEM - 1) / TILES_PER_ITEM;
        const u32 ri = (ne + RES_PER_ITEM - 1) / RES_PER_ITEM;
        if (q < p0) {
            d0 += di;
            r0 += ri;
        }
        d1 += di;
        r1 += ri;
    }
    SddmmArgs a = make_args(p, dA, dB, K, dP);
    a.d0 = d0;
    a.nd = d1 - d0;
    a.r0 = r0;
    a.nr = r1 - r0;
    return launch_panels(a, static_cast<hipStream_t>(stream));
}

extern "C" int bsmr_sddmm_panels_local(const bsmr_plan* plan, const void* dA_local,
                                       const void* dB, uint32_t K, int dtype, float* dP,
                                       uint32_t p0, uint32_t p1, void* stream) {
    if (!plan) {
        set_error("bsmr_sddmm_panels_local: null plan");
        return BSMR_ERR_INVALID;
    }
    const Plan& p = plan->p;
    BSMR_CHECK(validate(dA_local, dB, K, dtype, dP));
    if (p0 > p1 || p1 > p.P) {
        set_error("bsmr_sddmm_panels_local: bad panel range");
        return BSMR_ERR_INVALID;
    }
    if (p0 == p1) return BSMR_OK;
    const int slot = rb_slot(p, K, dtype);
    if (slot < 0) {
        set_error("bsmr_sddmm_panels_local: needs the row-block launch (rows of 128 B .. 2 KiB)");
        return BSMR_ERR_UNSUPPORTED;
    }
    {
        std::lock_guard<std::mutex> g(p.layout_mu);
        if (p.iotaR.size() < p.R) {
            std::vector<u32> id(p.R);
            for (u32 q = 0; q < p.R; ++q) id[q] = q;
            BSMR_CHECK(p.iotaR.upload(id.data(), p.R, p.stream));
            BSMR_HIP(hipStreamSynchronize(p.stream));
        }
    }
    std::shared_ptr<const Plan::RowBlockLayout> L;  // held until the launch is enqueued
    BSMR_CHECK(get_rb_layout(p, slot, dtype, p0, p1, &L));
    if (L->orig || L->cols)  // the whole range may have picked original-order row blocks or
                             // column blocks: use the reordered layout (always built first), whose
                             // rows follow the local A
        L = std::shared_ptr<const Plan::RowBlockLayout>(
            std::shared_ptr<void>(), &p.rbl[slot + (dtype != BSMR_F32 ? Plan::N_RB_SIZES : 0)]);
    return launch_rb(p, *L, dA_local, dB, dP, dtype, 3, static_cast<hipStream_t>(stream), 1, true);
}

extern "C" int bsmr_sddmm_profile(const bsmr_plan* plan, const void* dA, const void* dB,
                                  uint32_t K, int dtype, float* dP, int iters, void* stream,
                                  float* ms_dense, float* ms_residual, float* ms_total) {
    if (!plan || iters <= 0) {
        set_error("bsmr_sddmm_profile: bad arguments");
        return BSMR_ERR_INVALID;
    }
    const Plan& p = plan->p;
    BSMR_CHECK(validate(dA, dB, K, dtype, dP));
    hipStream_t s = static_cast<hipStream_t>(stream);
    struct Events {  // destroyed on every return path
        hipEvent_t e[4] = {};
        ~Events() {
            for (auto& x : e)
                if (x) (void)hipEventDestroy(x);
        }
    } evs;
    hipEvent_t* ev = evs.e;
    for (int i = 0; i < 4; ++i) BSMR_HIP(hipEventCreate(&ev[i]));
    const int slot = rb_slot(p, K, dtype);
    std::shared_ptr<const Plan::RowBlockLayout> L;
    if (slot >= 0 && !use_ptile(p, K, dtype)) BSMR_CHECK(get_rb_layout(p, slot, dtype, 0, p.P, &L));
    SddmmArgs full = make_args(p, dA, dB, K, dP);
    full.nd = p.nDenseItems;
    full.nslots = p.nSlots;
    SddmmArgs dense = full;
    dense.nslots = 0;
    SddmmArgs res = full;
    res.nd = 0;
    const bool ptile = use_ptile(p, K, dtype), dense_all = !ptile && use_dense(p, K, dtype);
    auto run = [&](u32 mode) -> int {
        if (ptile) return launch_ptile(p, dA, dB, K, dtype, dP, mode, s);
        if (dense_all) return launch_dense(p, dA, dB, K, dtype, dP, s);  // no dense/residual split
        if (L) return launch_rb(p, *L, dA, dB, dP, dtype, mode, s);
        if (dtype != BSMR_F32) return launch_half(p, dA, dB, K, dtype, dP, mode, s);
        return launch_full(p, mode == 1 ? dense : mode == 2 ? res : full, s);
    };
    BSMR_HIP(hipEventRecord(ev[0], s));
    for (int i = 0; i < iters; ++i) BSMR_CHECK(run(1));
    BSMR_HIP(hipEventRecord(ev[1], s));
    for (int i = 0; i < iters; ++i) BSMR_CHECK(run(2));
    BSMR_HIP(hipEventRecord(ev[2], s));
    for (int i = 0; i < iters; ++i) BSMR_CHECK(run(3));
    BSMR_HIP(hipEventRecord(ev[3], s));
    BSMR_HIP(hipEventSynchronize(ev[3]));
    float t0 = 0, t1 = 0, t2 = 0;
    BSMR_HIP(hipEventElapsedTime(&t0, ev[0], ev[1]));
    BSMR_HIP(hipEventElapsedTime(&t1, ev[1], ev[2]));
    BSMR_HIP(hipEventElapsedTime(&t2, ev[2], ev[3]));
    if (ms_dense) *ms_dense = p.nDenseItems ? t0 / iters : 0.f;
    if (ms_residual) *ms_residual = p.nres ? t1 / iters : 0.f;
    if (ms_total) *ms_total = t2 / iters;
    return BSMR_OK;
}

// debug: the whole-plan row-block layout of (K, dtype), 4 u32 per item slot in launch order
// {row block, kept tiles, entries, pieces} (padding slots all zero), preceded by the header
// {rows per block, threads per workgroup, items, row bytes}; *len = 4 (items + 1). Not in the
// header (tools/item_trace.py)
extern "C" int bsmr_debug_rb_items(const bsmr_plan* plan, uint32_t K, int dtype, uint32_t* host_out,
                                   uint64_t* len) {
    if (!plan) return BSMR_ERR_INVALID;
    const Plan& p = plan->p;
    const Plan::RowBlockLayout* L = nullptr;
    BSMR_CHECK(whole_rb_layout(p, K, dtype, &L));
    if (!L) {
        if (len) *len = 0;
        return BSMR_OK;
    }
    if (len) *len = 4ull * (L->itemStat.size() + 1);
    if (host_out) {
        host_out[0] = L->RB;
        host_out[1] = L->NT;
        host_out[2] = static_cast<uint32_t>(L->itemStat.size());
        host_out[3] = L->rowBytes;
        for (size_t i = 0; i < L->itemStat.size(); ++i) {
            const uint4 v = L->itemStat[i];
            host_out[4 * (i + 1) + 0] = v.x;
            host_out[4 * (i + 1) + 1] = v.y;
            host_out[4 * (i + 1) + 2] = v.z;
            host_out[4 * (i + 1) + 3] = v.w;
        }
    }
    return BSMR_OK;
}

// debug: the whole plan's row-block layout for (K, dtype) as {items (4 u32 each: row block, tile
// begin, tile end, piece begin), item ends, pieces (2 u32 each)}: *len = 4 n + n + 2 p + 2 with
// host_out[0] = n items, [1] = p pieces (tools/phase_balance.py; not in the header)
extern "C" int bsmr_debug_rb_pieces(const bsmr_plan* plan, uint32_t K, int dtype, uint32_t* host_out,
                                    uint64_t* len) {
    if (!plan) return BSMR_ERR_INVALID;
    const Plan& p = plan->p;
    const Plan::RowBlockLayout* L = nullptr;
    BSMR_CHECK(whole_rb_layout(p, K, dtype, &L));
    const u64 n = L ? L->nItems : 0, np = L ? L->nPieces : 0;
    if (len) *len = 2 + 5 * n + 2 * np;
    if (host_out && L) {
        host_out[0] = static_cast<uint32_t>(n);
        host_out[1] = static_cast<uint32_t>(np);
        BSMR_HIP(hipMemcpy(host_out + 2, L->items.data(), n * sizeof(uint4), hipMemcpyDeviceToHost));
        BSMR_HIP(hipMemcpy(host_out + 2 + 4 * n, L->itemEnd.data(), n * sizeof(u32), hipMemcpyDeviceToHost));
        BSMR_HIP(hipMemcpy(host_out + 2 + 5 * n, L->pieces.data(), np * sizeof(uint2), hipMemcpyDeviceToHost));
    }
    return BSMR_OK;
}

// debug timeline of the last traced launch (BSMR_DIAG & 32): 4 u64 per wave (not in the header)
extern "C" int bsmr_debug_trace(const bsmr_plan* plan, uint64_t* host_out, uint64_t* len) {
    if (!plan) return BSMR_ERR_INVALID;
    const Plan& p = plan->p;
    if (len) *len = p.traceN * 4ull;
    if (host_out && p.traceN) {
        BSMR_HIP(hipDeviceSynchronize());
        BSMR_HIP(hipMemcpy(host_out, p.trace.data(), p.traceN * 4ull * sizeof(uint64_t),
                           hipMemcpyDeviceToHost));
    }
    return BSMR_OK;
}
