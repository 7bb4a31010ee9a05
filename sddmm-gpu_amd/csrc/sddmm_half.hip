// sddmm_half.hip — SDDMM with fp16 / bf16 A and B, fp32 accumulation and fp32 P (configs C3
// cop20k_A fp16 K=256 and C5 DLMC bf16 K=512 of BASELINE.json; the reference builds TF32 only).
//
// Same plan, same launch structure as the fp32 column-major path (sddmm.hip):
//   * dense tile: `v_mfma_f32_16x16x32_{f16,bf16}`; lane l holds A[row l&15][32kk + 8(l>>4) + j]
//     and B[k = 32kk + 8(l>>4) + j][col l&15], j = 0..7 (one 16-byte load each); K/32 MFMAs.
//   * residual slot: one 16-lane row per entry, lane s holds W consecutive halves s, s+16, ... of
//     A[row] and B[col]; products of two halves are exact in fp32 and summed in fp32; DPP row sum.
#include <algorithm>

#include "common.hpp"
#include "plan.hpp"

namespace bsmr {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 b16x8 __attribute__((ext_vector_type(8)));

struct HalfArgs {
    const uint16_t* A;
    const uint16_t* B;
    float* P;
    u32 nd, nslots;
    const u32* tileRows;
    const u32* denseCols;
    const u32* blockValues;
    const uint2* slots;
    const u32* cmRow;
    const u32* cmCol;
    const u32* cmOut;
    u32 N, K;
    unsigned long long bA, bB, bP;  // batched launch (grid.y = batch), element strides
};

template <bool BF16>
__device__ __forceinline__ float h2f(uint16_t h) {
    if constexpr (BF16) {
        return __builtin_bit_cast(float, static_cast<u32>(h) << 16);
    } else {
        return static_cast<float>(__builtin_bit_cast(_Float16, h));
    }
}

template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                                 CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row_sum16(float v) {
    v += dppf<0xB1>(v);
    v += dppf<0x4E>(v);
    v += dppf<0x141>(v);
    v += dppf<0x140>(v);
    return v;
}

template <bool BF16>
__device__ __forceinline__ f32x4 mfma32(s16x8 a, s16x8 b, f32x4 c) {
    if constexpr (BF16)
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b16x8, a),
                                                       __builtin_bit_cast(b16x8, b), c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h16x8, a),
                                                      __builtin_bit_cast(h16x8, b), c, 0, 0, 0);
}

// one dense tile; K multiple of 32
template <bool BF16>
__device__ __forceinline__ void dense_tile_h(const HalfArgs& a, const u32 tile) {
    const u32 l = __lane_id(), rr = l & 15, g = l >> 4;
    const u32 row = a.tileRows[tile * 16 + rr];
    const u32 c = a.denseCols[tile * 16 + rr];
    const u32* bvals = a.blockValues + static_cast<size_t>(tile) * 256 + 64 * g + rr;
    u32 idx[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) idx[r] = bvals[16 * r];
    const bool rvalid = row != NULLV;
    const bool cvalid = c < a.N;
    const uint16_t* arow = a.A + static_cast<size_t>(rvalid ? row : 0) * a.K + 8 * g;
    const uint16_t* bcol = a.B + static_cast<size_t>(cvalid ? c : 0) * a.K + 8 * g;
    f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
    const s16x8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
    u32 k = 0;
    for (; k + 64 <= a.K; k += 64) {
        const s16x8 a0 = rvalid ? *reinterpret_cast<const s16x8*>(arow + k) : zero;
        const s16x8 b0 = cvalid ? *reinterpret_cast<const s16x8*>(bcol + k) : zero;
        const s16x8 a1 = rvalid ? *reinterpret_cast<const s16x8*>(arow + k + 32) : zero;
        const s16x8 b1 = cvalid ? *reinterpret_cast<const s16x8*>(bcol + k + 32) : zero;
        acc0 = mfma32<BF16>(a0, b0, acc0);
        acc1 = mfma32<BF16>(a1, b1, acc1);
    }
    if (k < a.K) {
        const s16x8 a0 = rvalid ? *reinterpret_cast<const s16x8*>(arow + k) : zero;
        const s16x8 b0 = cvalid ? *reinterpret_cast<const s16x8*>(bcol + k) : zero;
        acc0 = mfma32<BF16>(a0, b0, acc0);
    }
    const f32x4 acc = acc0 + acc1;
#pragma unroll
    for (int r = 0; r < 4; ++r)
        if (idx[r] != NULLV) a.P[idx[r]] = acc[r];
}

// residual slot: each 16-lane row takes a contiguous share; lane s reads 2 halves (4 bytes) at
// k = 2s + 32j, j = 0 .. K/32-1, for A and B; up to U entries in flight per row
template <bool BF16>
__device__ __forceinline__ void residual_h(const HalfArgs& a, const uint2 sl) {
    constexpr int U = 4;
    const u32 l = __lane_id(), sub = l & 15, grp = l >> 4;
    const u32 n = sl.y - sl.x;
    const u32 share = (n + 3) / 4;
    const u32 gs = sl.x + min(grp * share, n), ge = sl.x + min(grp * share + share, n);
    const u32 K = a.K;
    for (u32 base = gs; base < ge; base += U) {
        float acc[U];
        u32 out[U];
        bool ok[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u32 e = base + u;
            ok[u] = e < ge;
            const u32 ee = ok[u] ? e : gs;
            out[u] = a.cmOut[ee];
            const uint16_t* ap = a.A + static_cast<size_t>(a.cmRow[ee]) * K + 2 * sub;
            const uint16_t* bp = a.B + static_cast<size_t>(a.cmCol[ee]) * K + 2 * sub;
            float s = 0.f;
            for (u32 k = 0; k < K; k += 32) {
                const u32 av = *reinterpret_cast<const u32*>(ap + k);
                const u32 bv = *reinterpret_cast<const u32*>(bp + k);
                s += h2f<BF16>(static_cast<uint16_t>(av)) * h2f<BF16>(static_cast<uint16_t>(bv));
                s += h2f<BF16>(static_cast<uint16_t>(av >> 16)) *
                     h2f<BF16>(static_cast<uint16_t>(bv >> 16));
            }
            acc[u] = s;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float t = row_sum16(acc[u]);
            if (sub == 0 && ok[u]) a.P[out[u]] = t;
        }
    }
}

template <bool BF16>
__global__ __launch_bounds__(64) void k_sddmm_half(HalfArgs a) {
    if (blockIdx.y) {
        a.A += blockIdx.y * a.bA;
        a.B += blockIdx.y * a.bB;
        a.P += blockIdx.y * a.bP;
    }
    const u32 b = blockIdx.x;
    if (b < a.nd) {
        dense_tile_h<BF16>(a, b);
        return;
    }
    const u32 ndpad = (a.nd + 7) & ~7u;
    if (b < ndpad) return;
    const u32 s = b - ndpad;
    if (s < a.nslots) {
        const uint2 sl = a.slots[s];
        if (sl.x < sl.y) residual_h<BF16>(a, sl);
    }
}

}  // namespace

// dtype: BSMR_F16 or BSMR_BF16; K a positive multiple of 32. mode: 1 dense, 2 residual, 3 both
int launch_half(const Plan& p, const void* dA, const void* dB, u32 K, int dtype, float* dP,
                u32 mode, hipStream_t s, u32 nb) {
    if (K == 0 || K % 32 != 0) {
        set_error("bsmr_sddmm: fp16/bf16 inputs need K to be a positive multiple of 32");
        return BSMR_ERR_UNSUPPORTED;
    }
    HalfArgs a{};
    a.A = static_cast<const uint16_t*>(dA);
    a.B = static_cast<const uint16_t*>(dB);
    a.P = dP;
    a.nd = (mode & 1) ? p.nDenseItems : 0;
    a.nslots = (mode & 2) ? p.nSlots : 0;
    a.tileRows = p.tileRows.data();
    a.denseCols = p.denseCols.data();
    a.blockValues = p.blockValues.data();
    a.slots = p.cmSlots.data();
    a.cmRow = p.cmRow.data();
    a.cmCol = p.cmCol.data();
    a.cmOut = p.cmOut.data();
    a.N = p.N;
    a.K = K;
    a.bA = static_cast<unsigned long long>(p.M) * K;
    a.bB = static_cast<unsigned long long>(p.N) * K;
    a.bP = p.nnz;
    const u32 grid = a.nslots ? ((a.nd + 7) & ~7u) + a.nslots : a.nd;
    if (grid == 0) return BSMR_OK;
    if (dtype == BSMR_BF16)
        hipLaunchKernelGGL(k_sddmm_half<true>, dim3(grid, nb), dim3(64), 0, s, a);
    else
        hipLaunchKernelGGL(k_sddmm_half<false>, dim3(grid, nb), dim3(64), 0, s, a);
    BSMR_HIP(hipGetLastError());
    return BSMR_OK;
}

}  // namespace bsmr
