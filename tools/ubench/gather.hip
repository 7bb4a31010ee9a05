// Microbenchmark: cost of 16-byte-per-lane gathers of 512-byte rows (one row per 4-lane group)
// under partial exec masks, from an L2/MALL-resident table; and dependent-step latency.
// hipcc --offload-arch=gfx950 -O3 -o gather gather.hip && ./gather
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

// each wave: S steps; per step every 4-lane group whose (hash & mask) == 0 loads its row's
// 8 chunks (512 B per group), then all lanes fold the data into an accumulator
template <int S>
__global__ __launch_bounds__(1024) void k_gather(const float* __restrict__ B, unsigned nrows,
                                                 unsigned mask, unsigned same, float* out) {
    const unsigned tid = threadIdx.x, grp = (blockIdx.x * 1024 + tid) >> 2, sub = tid & 3;
    f4 acc = {0, 0, 0, 0};
    f4 bv[8];
    for (int f = 0; f < 8; ++f) bv[f] = f4{0, 0, 0, 0};
    unsigned h = grp * 2654435761u;
#pragma unroll 1
    for (int s = 0; s < S; ++s) {
        h = h * 1664525u + 1013904223u;
        const unsigned row = same ? (blockIdx.x * 7 + s) % nrows : (h >> 8) % nrows;
        if (((h >> 3) & mask) == 0) {
            const char* p = reinterpret_cast<const char*>(B) + (size_t)row * 512 + 16 * sub;
#pragma unroll
            for (int f = 0; f < 8; ++f) bv[f] = *reinterpret_cast<const f4*>(p + 64 * f);
        }
#pragma unroll
        for (int f = 0; f < 8; ++f) acc += bv[f];
        h ^= __float_as_uint(acc.x) & 1u;  // make the next step depend on this one
    }
    if (acc.x + acc.y + acc.z + acc.w == 1234.5f) out[0] = acc.x;
}

int main() {
    const unsigned nrows = 12419;  // 6.4 MB of 512-byte rows (C2's B at K = 128)
    float *B, *out;
    hipMalloc(&B, (size_t)nrows * 512);
    hipMalloc(&out, 64);
    hipMemset(B, 0, (size_t)nrows * 512);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const unsigned masks[] = {0, 1, 3, 7, 15, 0xFFFFFFFF};
    for (unsigned same = 0; same < 2; ++same)
        for (unsigned m : masks) {
            for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k_gather<8>, dim3(256), dim3(1024), 0, 0, B, nrows, m, same, out);
            hipEventRecord(e0);
            for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(k_gather<8>, dim3(256), dim3(1024), 0, 0, B, nrows, m, same, out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double frac = m == 0xFFFFFFFF ? 0.0 : 1.0 / (m + 1);
            const double bytes = 256.0 * 256 * 8 * 512 * frac;  // groups * steps * 512 B * active
            printf("{\"same\": %u, \"active_frac\": %.4f, \"us\": %.2f, \"GBps_active\": %.0f}\n", same,
                   frac, ms * 1000 / 20, bytes / (ms / 20 * 1e-3) / 1e9);
        }
    // 1 step vs 8 steps: dependent-step latency
    for (int S : {1, 8}) {
        auto fn = S == 1 ? k_gather<1> : k_gather<8>;
        for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(fn, dim3(256), dim3(1024), 0, 0, B, nrows, 0u, 0u, out);
        hipEventRecord(e0);
        for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(fn, dim3(256), dim3(1024), 0, 0, B, nrows, 0u, 0u, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("{\"steps\": %d, \"us\": %.2f}\n", S, ms * 1000 / 20);
    }
    return 0;
}
