// Launch floor of back-to-back SDDMM-shaped launches: kernels that do nothing (or one 16-byte
// load per lane, one dependent round trip) with the product launches' geometry (256 workgroups of
// 1024 / 512 threads, 0-160 KiB of LDS), 200 per HIP graph, timed between HIP events. The
// difference between a product kernel's step time and this floor is its own work.
//   hipcc --offload-arch=gfx950 -O3 -o launch_floor launch_floor.hip && ./launch_floor
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                          \
        }                                                                          \
    } while (0)

template <int NT>
__global__ __launch_bounds__(NT) void k_nop(const float4* src, float* sink, int load) {
    extern __shared__ float lds[];
    if (load) {
        const float4 v = src[blockIdx.x * NT + threadIdx.x];
        if (v.x == -1234.5f) sink[threadIdx.x] = v.y + lds[threadIdx.x];  // never
    }
}

template <int NT>
static float time_graph(int grid, size_t lds, int load, const float4* src, float* sink, int steps) {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_nop<NT>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < steps; ++i) hipLaunchKernelGGL(k_nop<NT>, dim3(grid), dim3(NT), lds, s, src, sink, load);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int r = 0; r < 4; ++r) {
        CK(hipGraphLaunch(ge, s));  // r = 0: warm-up
        CK(hipEventRecord(e0, s));
        CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(e1, s));
        CK(hipStreamSynchronize(s));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r > 0 && ms < best) best = ms;
    }
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    CK(hipStreamDestroy(s));
    return best * 1e3f / steps;  // us per launch
}

int main() {
    const int steps = 200;
    float4* src;
    float* sink;
    CK(hipMalloc(&src, sizeof(float4) * 1024 * 1024));
    CK(hipMemset(src, 0, sizeof(float4) * 1024 * 1024));
    CK(hipMalloc(&sink, 4096));
    std::printf("{\"steps\": %d, \"rows\": [\n", steps);
    const int grids[] = {256, 512, 1024};
    const size_t ldss[] = {0, 64 * 1024, 160 * 1024};
    bool first = true;
    for (int load = 0; load < 2; ++load)
        for (int nt = 0; nt < 2; ++nt)
            for (int gi = 0; gi < 3; ++gi)
                for (int li = 0; li < 3; ++li) {
                    const int grid = grids[gi];
                    if (grid * (nt ? 1024 : 512) > 1024 * 1024) continue;
                    const float us = nt ? time_graph<1024>(grid, ldss[li], load, src, sink, steps)
                                        : time_graph<512>(grid, ldss[li], load, src, sink, steps);
                    std::printf("%s  {\"threads\": %d, \"grid\": %d, \"lds_kb\": %zu, \"load\": %d, \"us\": %.3f}",
                                first ? "" : ",\n", nt ? 1024 : 512, grid, ldss[li] / 1024, load, us);
                    first = false;
                }
    std::printf("\n]}\n");
    CK(hipFree(src));
    CK(hipFree(sink));
    return 0;
}
