// sddmm.hip — the SDDMM launch over a BSMR plan (gfx950, wave64, MFMA).
//
// One launch, one wave per work item (64-thread workgroups):
//   * dense item  {panel, first tile, ntiles}: the panel's 16 A rows stay in registers (KT/4 VGPRs)
//     and each 16x16 tile is 4*K/16 `v_mfma_f32_16x16x4_f32` (exact fp32, no TF32 on gfx950).
//     Lane l holds A[row l&15][16kk + 4(l>>4) + e] and B[col l&15][same k]; instruction e of
//     step kk therefore sums k = 16kk + 4g + e over the four lane groups g, covering every k once.
//     Accumulator lane l, reg r = D[4(l>>4)+r][l&15], scattered through blockValues
//     (replaces sddmm_gpu_dense_block_m16n16k8_*, sddmmKernel.cu:213-351, 355-488).
//   * residual item {panel, e0, e1}: the panel's A rows staged in LDS (row stride K+4), G lanes
//     per entry read 16 B of B each (a G*16-byte coalesced piece of the column), fp32 FMA, xor
//     shuffle reduction (replaces sddmm_gpu_sparse_*_2threadOneData_shuffle,
//     sddmmKernel.cu:1994-2104, 2109-2199).
// The reference launches a panels x ceil(maxBlocks/4) dense grid and a second kernel on another
// stream; the compact item lists make both parts one dense, balanced grid.
#include <algorithm>
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
    const uint4* ditems;
    const uint4* ritems;
    u32 d0, nd;  // dense items [d0, d0+nd)
    u32 r0, nr;  // residual items [r0, r0+nr)
    const u32* rows;
    u32 R, N, K;
    const u32* denseCols;
    const u32* blockValues;
    const u32* sparseValues;
    const u32* sparseRel;
    const u32* sparseCol;
};

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

// dense tiles, K = KT known at compile time (A panel cached in registers)
template <int KT>
__device__ __forceinline__ void dense_item(const SddmmArgs& a, const uint4 it) {
    constexpr int NK = KT / 16;
    const u32 l = __lane_id(), rr = l & 15, g = l >> 4;
    const u32 q = it.x * 16 + rr;
    const bool rvalid = q < a.R;
    const float* arow = a.A + static_cast<size_t>(rvalid ? a.rows[q] : 0) * KT + 4 * g;
    f32x4 av[NK];
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) av[kk] = rvalid ? ld4(arow + 16 * kk) : f32x4{0, 0, 0, 0};
    for (u32 t = 0; t < it.z; ++t) {
        const u32 tile = it.y + t;
        const u32 c = a.denseCols[tile * 16 + rr];
        const bool cvalid = c < a.N;
        const float* bcol = a.B + static_cast<size_t>(cvalid ? c : 0) * KT + 4 * g;
        f32x4 acc = {0, 0, 0, 0};
#pragma unroll
        for (int kk = 0; kk < NK; ++kk) {
            const f32x4 bv = cvalid ? ld4(bcol + 16 * kk) : f32x4{0, 0, 0, 0};
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kk].x, bv.x, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kk].y, bv.y, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kk].z, bv.z, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kk].w, bv.w, acc, 0, 0, 0);
        }
        const u32* bvals = a.blockValues + static_cast<size_t>(tile) * 256 + 64 * g + rr;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const u32 idx = bvals[16 * r];
            if (idx != NULLV) a.P[idx] = acc[r];
        }
    }
}

// dense tiles, runtime K (multiple of 16): A re-read per tile
__device__ __forceinline__ void dense_item_generic(const SddmmArgs& a, const uint4 it) {
    const u32 l = __lane_id(), rr = l & 15, g = l >> 4;
    const u32 q = it.x * 16 + rr;
    const bool rvalid = q < a.R;
    const float* arow = a.A + static_cast<size_t>(rvalid ? a.rows[q] : 0) * a.K + 4 * g;
    for (u32 t = 0; t < it.z; ++t) {
        const u32 tile = it.y + t;
        const u32 c = a.denseCols[tile * 16 + rr];
        const bool cvalid = c < a.N;
        const float* bcol = a.B + static_cast<size_t>(cvalid ? c : 0) * a.K + 4 * g;
        f32x4 acc = {0, 0, 0, 0};
        for (u32 k = 0; k < a.K; k += 16) {
            const f32x4 av = rvalid ? ld4(arow + k) : f32x4{0, 0, 0, 0};
            const f32x4 bv = cvalid ? ld4(bcol + k) : f32x4{0, 0, 0, 0};
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bv.x, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, bv.y, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, bv.z, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, bv.w, acc, 0, 0, 0);
        }
        const u32* bvals = a.blockValues + static_cast<size_t>(tile) * 256 + 64 * g + rr;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const u32 idx = bvals[16 * r];
            if (idx != NULLV) a.P[idx] = acc[r];
        }
    }
}

// residual entries: G lanes per entry
template <int G>
__device__ __forceinline__ void residual_item(const SddmmArgs& a, const uint4 it, float* As) {
    const u32 l = __lane_id();
    const u32 K = a.K, KP = K + 4;
    // stage the panel's 16 A rows (zeros past the last reordered row)
    for (u32 x = 4 * l; x < 16 * K; x += 256) {
        const u32 r = x / K, k = x - r * K;
        const u32 q = it.x * 16 + r;
        const f32x4 v = q < a.R ? ld4(a.A + static_cast<size_t>(a.rows[q]) * K + k) : f32x4{0, 0, 0, 0};
        *reinterpret_cast<f32x4*>(As + r * KP + k) = v;
    }
    __syncthreads();
    constexpr u32 EPI = 64 / G;
    const u32 sub = l % G, grp = l / G;
    for (u32 e = it.y + grp; e < it.z; e += EPI) {
        const u32 rr = a.sparseRel[e];
        const u32 c = a.sparseCol[e];
        const float* brow = a.B + static_cast<size_t>(c) * K;
        const float* arow = As + rr * KP;
        float acc = 0.f;
        for (u32 k = 4 * sub; k < K; k += 4 * G) {
            const f32x4 av = *reinterpret_cast<const f32x4*>(arow + k);
            const f32x4 bv = ld4(brow + k);
            acc += av.x * bv.x + av.y * bv.y + av.z * bv.z + av.w * bv.w;
        }
#pragma unroll
        for (int o = G / 2; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
        if (sub == 0) a.P[a.sparseValues[e]] = acc;
    }
    __syncthreads();
}

template <int KT, int G>
__global__ __launch_bounds__(64) void k_sddmm_f32(SddmmArgs a) {
    extern __shared__ __attribute__((aligned(16))) float As[];
    const u32 b = blockIdx.x;
    if (b < a.nd) {
        const uint4 it = a.ditems[a.d0 + b];
        if constexpr (KT > 0)
            dense_item<KT>(a, it);
        else
            dense_item_generic(a, it);
    } else {
        const u32 rb = b - a.nd;
        if (rb < a.nr) residual_item<G>(a, a.ritems[a.r0 + rb], As);
    }
}

using KernelFn = void (*)(SddmmArgs);

template <int G>
KernelFn pick_k(u32 K) {
    switch (K) {
        case 32: return k_sddmm_f32<32, G>;
        case 64: return k_sddmm_f32<64, G>;
        case 128: return k_sddmm_f32<128, G>;
        case 256: return k_sddmm_f32<256, G>;
        case 512: return k_sddmm_f32<512, G>;
        default: return k_sddmm_f32<0, G>;
    }
}

KernelFn pick_kernel(u32 K) {
    if (K % 64 == 0) return pick_k<16>(K);
    if (K % 32 == 0) return pick_k<8>(K);
    return pick_k<4>(K);
}

int validate(const Plan& p, const void* dA, const void* dB, u32 K, int dtype, const float* dP) {
    if (!dA || !dB || !dP) {
        set_error("bsmr_sddmm: null device pointer");
        return BSMR_ERR_INVALID;
    }
    if (K == 0 || K % 16 != 0) {
        set_error("bsmr_sddmm: K must be a positive multiple of 16");
        return BSMR_ERR_UNSUPPORTED;
    }
    if (dtype != BSMR_F32) {
        set_error("bsmr_sddmm: this build supports fp32 A/B only");
        return BSMR_ERR_UNSUPPORTED;
    }
    (void)p;
    return BSMR_OK;
}

SddmmArgs make_args(const Plan& p, const void* dA, const void* dB, u32 K, float* dP) {
    SddmmArgs a{};
    a.A = static_cast<const float*>(dA);
    a.B = static_cast<const float*>(dB);
    a.P = dP;
    a.ditems = p.denseItems.data();
    a.ritems = p.resItems.data();
    a.rows = p.rows.data();
    a.R = p.R;
    a.N = p.N;
    a.K = K;
    a.denseCols = p.denseCols.data();
    a.blockValues = p.blockValues.data();
    a.sparseValues = p.sparseValues.data();
    a.sparseRel = p.sparseRel.data();
    a.sparseCol = p.sparseColIdx.data();
    return a;
}

size_t lds_bytes(u32 K) { return static_cast<size_t>(16) * (K + 4) * sizeof(float); }

int launch(const Plan& p, SddmmArgs a, hipStream_t s) {
    const u32 grid = a.nd + a.nr;
    if (grid == 0) return BSMR_OK;
    hipLaunchKernelGGL(pick_kernel(a.K), dim3(grid), dim3(64), a.nr ? lds_bytes(a.K) : 0, s, a);
    BSMR_HIP(hipGetLastError());
    (void)p;
    return BSMR_OK;
}

// item ranges of the panels [p0, p1): items are stored panel-major
void item_range(const std::vector<u32>& off_per_panel, u32 p0, u32 p1, u32& i0, u32& i1) {
    i0 = off_per_panel[p0];
    i1 = off_per_panel[p1];
}

}  // namespace
}  // namespace bsmr

using namespace bsmr;

extern "C" int bsmr_sddmm(const bsmr_plan* plan, const void* dA, const void* dB, uint32_t K,
                          int dtype, float* dP, void* stream) {
    if (!plan) {
        set_error("bsmr_sddmm: null plan");
        return BSMR_ERR_INVALID;
    }
    const Plan& p = plan->p;
    BSMR_CHECK(validate(p, dA, dB, K, dtype, dP));
    SddmmArgs a = make_args(p, dA, dB, K, dP);
    a.d0 = 0;
    a.nd = p.nDenseItems;
    a.r0 = 0;
    a.nr = p.nResItems;
    return launch(p, a, static_cast<hipStream_t>(stream));
}

extern "C" int bsmr_sddmm_panels(const bsmr_plan* plan, const void* dA, const void* dB,
                                 uint32_t K, int dtype, float* dP, uint32_t p0, uint32_t p1,
                                 void* stream) {
    if (!plan) {
        set_error("bsmr_sddmm_panels: null plan");
        return BSMR_ERR_INVALID;
    }
    const Plan& p = plan->p;
    BSMR_CHECK(validate(p, dA, dB, K, dtype, dP));
    if (p0 > p1 || p1 > p.P) {
        set_error("bsmr_sddmm_panels: bad panel range");
        return BSMR_ERR_INVALID;
    }
    // dense items of panel q: ceil(tiles_q / TILES_PER_ITEM); residual: ceil(nres_q / RES_PER_ITEM)
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
    return launch(p, a, static_cast<hipStream_t>(stream));
}

extern "C" int bsmr_sddmm_profile(const bsmr_plan* plan, const void* dA, const void* dB,
                                  uint32_t K, int dtype, float* dP, int iters, void* stream,
                                  float* ms_dense, float* ms_residual, float* ms_total) {
    if (!plan || iters <= 0) {
        set_error("bsmr_sddmm_profile: bad arguments");
        return BSMR_ERR_INVALID;
    }
    const Plan& p = plan->p;
    BSMR_CHECK(validate(p, dA, dB, K, dtype, dP));
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipEvent_t ev[6];
    for (auto& e : ev) BSMR_HIP(hipEventCreate(&e));
    SddmmArgs full = make_args(p, dA, dB, K, dP);
    full.nd = p.nDenseItems;
    full.nr = p.nResItems;
    SddmmArgs dense = full;
    dense.nr = 0;
    SddmmArgs res = full;
    res.nd = 0;
    BSMR_HIP(hipEventRecord(ev[0], s));
    for (int i = 0; i < iters; ++i) BSMR_CHECK(launch(p, dense, s));
    BSMR_HIP(hipEventRecord(ev[1], s));
    for (int i = 0; i < iters; ++i) BSMR_CHECK(launch(p, res, s));
    BSMR_HIP(hipEventRecord(ev[2], s));
    for (int i = 0; i < iters; ++i) BSMR_CHECK(launch(p, full, s));
    BSMR_HIP(hipEventRecord(ev[3], s));
    BSMR_HIP(hipEventSynchronize(ev[3]));
    float t0 = 0, t1 = 0, t2 = 0;
    BSMR_HIP(hipEventElapsedTime(&t0, ev[0], ev[1]));
    BSMR_HIP(hipEventElapsedTime(&t1, ev[1], ev[2]));
    BSMR_HIP(hipEventElapsedTime(&t2, ev[2], ev[3]));
    if (ms_dense) *ms_dense = p.nDenseItems ? t0 / iters : 0.f;
    if (ms_residual) *ms_residual = p.nResItems ? t1 / iters : 0.f;
    if (ms_total) *ms_total = t2 / iters;
    for (auto& e : ev) (void)hipEventDestroy(e);
    return BSMR_OK;
}
