// Shader clock across a run of back-to-back launches from a standing start: each launch's first
// wave reads s_memtime (shader clock cycles) and s_memrealtime (100 MHz) at its start and after a
// fixed amount of ALU work; cycles / real ticks = the clock the launch ran at. 400 launches of a
// ~10 us kernel (256 workgroups x 1024 threads, as the C2 launch) in one HIP graph, after the
// device sat idle for a second.
//   hipcc --offload-arch=gfx950 -O3 -o clock_ramp clock_ramp.hip && ./clock_ramp
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#define CK(x)                                                                                    \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
            std::exit(1);                                                                        \
        }                                                                                        \
    } while (0)

__global__ __launch_bounds__(1024) void k_spin(unsigned long long* out, int launch, int iters) {
    unsigned long long c0 = 0, r0 = 0;
    const bool rec = blockIdx.x == 0 && threadIdx.x == 0;
    if (rec) {
        c0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    float x = threadIdx.x * 1e-3f, y = 1.0001f;
    for (int i = 0; i < iters; ++i) x = __builtin_fmaf(x, y, 1e-7f);
    if (rec) {
        const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        out[4 * launch + 0] = c1 - c0;
        out[4 * launch + 1] = r1 - r0;
        out[4 * launch + 2] = r0;
        out[4 * launch + 3] = x == -1.f ? 1 : 0;  // keeps the loop
    }
}

int main() {
    const int n = 400, iters = 4000;
    unsigned long long* d;
    CK(hipMalloc(&d, sizeof(unsigned long long) * 4 * n));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_spin, dim3(256), dim3(1024), 0, s, d, i, iters);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    std::printf("{\"launches\": %d, \"runs\": [\n", n);
    for (int run = 0; run < 2; ++run) {
        std::this_thread::sleep_for(std::chrono::milliseconds(1000));  // a standing start
        CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        std::vector<unsigned long long> h(4 * n);
        CK(hipMemcpy(h.data(), d, sizeof(unsigned long long) * 4 * n, hipMemcpyDeviceToHost));
        std::printf("%s  {\"mhz\": [", run ? ",\n" : "");
        for (int i = 0; i < n; ++i)
            std::printf("%s%.0f", i ? ", " : "", h[4 * i + 1] ? 100.0 * h[4 * i] / h[4 * i + 1] : 0.0);
        std::printf("], \"t_us\": [");
        for (int i = 0; i < n; ++i) std::printf("%s%.1f", i ? ", " : "", (h[4 * i + 2] - h[2]) / 100.0);
        std::printf("]}");
    }
    std::printf("\n]}\n");
    return 0;
}
