// host_check.cpp — the reference's validation path as product code (not the test oracle):
// host SDDMM (src/host.cpp:45-76) and checkData (include/checkData.hpp:14-96), used by the
// BSMR-sddmm validate switch (BSMR_VALIDATE=1, the reference's `#define VALIDATE`,
// src/sddmm.cu:7,34-59) and exported through the C ABI (include/bsmr.h).
//
// Compiled with -ffp-contract=off: every output is a serial fp32 `val += a * b` over k ascending,
// as the reference's g++ -O3 x86-64 build computes it (SSE, no FMA, no reassociation), so the
// values do not depend on the thread count.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <thread>
#include <vector>

#include "common.hpp"

namespace {

void sddmm_rows(const uint32_t* rowptr, const uint32_t* colidx, uint32_t K, const float* A,
                const float* B, float* P, uint32_t r0, uint32_t r1) {
    for (uint32_t row = r0; row < r1; ++row) {
        const float* a = A + static_cast<size_t>(row) * K;
        for (uint32_t idx = rowptr[row]; idx < rowptr[row + 1]; ++idx) {
            const float* b = B + static_cast<size_t>(colidx[idx]) * K;
            float val = 0.0f;
            for (uint32_t k = 0; k < K; ++k) val += a[k] * b[k];
            P[idx] = val;
        }
    }
}

}  // namespace

// sddmm_cpu (host.cpp:45-76): the reference parallelises rows with `omp parallel for`; rows
// are cut here into contiguous, equal-entry ranges over std::threads (same per-entry values)
extern "C" int bsmr_sddmm_cpu(const uint32_t* rowptr, const uint32_t* colidx, uint32_t M,
                              uint32_t N, uint32_t K, const float* A, const float* B, float* P,
                              int nthreads) {
    if (!rowptr || !colidx || !A || !B || !P || M == 0 || N == 0 || K == 0) {
        bsmr::set_error("bsmr_sddmm_cpu: bad arguments");
        return BSMR_ERR_INVALID;
    }
    const uint64_t nnz = rowptr[M];
    for (uint64_t i = 0; i < nnz; ++i)
        if (colidx[i] >= N) {
            bsmr::set_error("bsmr_sddmm_cpu: column index out of range");
            return BSMR_ERR_INVALID;
        }
    unsigned T = nthreads > 0 ? static_cast<unsigned>(nthreads)
                              : std::max(1u, std::thread::hardware_concurrency());
    T = std::min<unsigned>(T, M);
    if (T <= 1) {
        sddmm_rows(rowptr, colidx, K, A, B, P, 0, M);
        return BSMR_OK;
    }
    // cut points by stored entries (+1 per row), so power-law rows do not serialise one thread
    std::vector<uint32_t> cut(T + 1, M);
    cut[0] = 0;
    const double total = static_cast<double>(nnz) + M;
    uint32_t r = 0;
    for (unsigned t = 1; t < T; ++t) {
        const double target = total * t / T;
        while (r < M && static_cast<double>(rowptr[r]) + r < target) ++r;
        cut[t] = r;
    }
    std::vector<std::thread> pool;
    pool.reserve(T);
    for (unsigned t = 0; t < T; ++t)
        if (cut[t] < cut[t + 1])
            pool.emplace_back(sddmm_rows, rowptr, colidx, K, A, B, P, cut[t], cut[t + 1]);
    for (auto& th : pool) th.join();
    return BSMR_OK;
}

// checkOneData<float> (checkData.hpp:21-30)
extern "C" int bsmr_check_one(float data1, float data2) {
    constexpr float ABS_EPSILON = 1e-5f;
    constexpr float EPS = 1e-3f;  // ERROR_THRESHOLD_EPSILON (checkData.hpp:14)
    const float absDiff = std::fabs(data1 - data2);
    if (absDiff < ABS_EPSILON) return 1;
    const float maxVal = std::max(std::max(std::fabs(data1), std::fabs(data2)), EPS);
    return (absDiff / maxVal) < EPS ? 1 : 0;
}

// checkDataFunction (checkData.hpp:44-79): the framed report on stdout when verbose, the first
// nine mismatches, and the number of mismatches as the return value
extern "C" uint64_t bsmr_check_data(uint64_t n, const float* data1, const float* data2,
                                    int verbose) {
    if (verbose) {
        std::printf("|---------------------------check data---------------------------|\n");
        std::printf("| Data size : %ld\n", static_cast<long>(n));
        std::printf("| Error threshold epsilon : %f\n", static_cast<double>(1e-3f));
        std::printf("| Checking results...\n");
    }
    uint64_t errors = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if (bsmr_check_one(data1[i], data2[i])) continue;
        ++errors;
        if (verbose && errors < 10)
            std::printf("| Error : idx = %d, data1 = %f, data2 = %f, difference = %f\n",
                        static_cast<int>(i), static_cast<double>(data1[i]),
                        static_cast<double>(data2[i]), static_cast<double>(data1[i] - data2[i]));
    }
    if (verbose) {
        if (errors > 0)
            std::printf("| No Pass! Inconsistent data! %zu errors! Error rate : %2.2f%%\n",
                        static_cast<size_t>(errors),
                        static_cast<double>(static_cast<float>(errors) / static_cast<float>(n) * 100));
        else
            std::printf("| Pass! Result validates successfully.\n");
        std::printf("|----------------------------------------------------------------|\n");
        std::fflush(stdout);
    }
    return errors;
}
