// rocSPARSE SDDMM baseline (include/bsmr_rocsparse.h). The counterpart of the reference's
// cuSPARSE baseline (include/cuSparseSDDMM.cuh:27-145): same operands, alpha = 1, beta = 0,
// default algorithm, buffer_size + preprocess once, then one rocsparse_sddmm per call.
#include "bsmr_rocsparse.h"

#include <hip/hip_runtime.h>
#include <rocsparse/rocsparse.h>

#include <cstdio>
#include <string>

namespace {

thread_local std::string g_err;

int fail(const char* what, int code) {
    g_err = what;
    return code;
}

// bsmr_status codes (include/bsmr.h)
constexpr int kOk = 0, kInvalid = 1, kHip = 4, kUnsupported = 6;

}  // namespace

struct bsmr_rocsparse {
    rocsparse_handle handle = nullptr;
    rocsparse_dnmat_descr A = nullptr, B = nullptr;
    rocsparse_spmat_descr C = nullptr;
    rocsparse_datatype ab_type = rocsparse_datatype_f32_r;
    rocsparse_sddmm_alg alg = rocsparse_sddmm_alg_default;
    void* buffer = nullptr;
    float* scratch = nullptr;  // C values bound during preprocess
    float alpha = 1.0f, beta = 0.0f;
};

#define RS_CHECK(call)                                                                   \
    do {                                                                                 \
        rocsparse_status s_ = (call);                                                    \
        if (s_ != rocsparse_status_success) {                                            \
            char m_[320];                                                                \
            std::snprintf(m_, sizeof m_, "rocsparse_status %d %s (%s) in %.120s", (int)s_,     \
                          rocsparse_get_status_name(s_),                                 \
                          rocsparse_get_status_description(s_), #call);                  \
            g_err = m_;                                                                  \
            return kHip;                                                                 \
        }                                                                                \
    } while (0)

extern "C" {

const char* bsmr_rocsparse_last_error(void) { return g_err.c_str(); }

void bsmr_rocsparse_destroy(bsmr_rocsparse* h) {
    if (!h) return;
    if (h->buffer) (void)hipFree(h->buffer);
    if (h->scratch) (void)hipFree(h->scratch);
    if (h->A) rocsparse_destroy_dnmat_descr(h->A);
    if (h->B) rocsparse_destroy_dnmat_descr(h->B);
    if (h->C) rocsparse_destroy_spmat_descr(h->C);
    if (h->handle) rocsparse_destroy_handle(h->handle);
    delete h;
}

static int create_impl(bsmr_rocsparse* h, uint32_t M, uint32_t N, uint32_t K, uint32_t nnz,
                       const uint32_t* d_rowptr, const uint32_t* d_colidx, void* stream) {
    RS_CHECK(rocsparse_create_handle(&h->handle));
    RS_CHECK(rocsparse_set_stream(h->handle, (hipStream_t)stream));
    // Values are bound per call (rocsparse_dnmat_set_values / rocsparse_spmat_set_values); the
    // descriptors need non-null pointers for preprocess, which reads only the pattern.
    void* dummy = (void*)d_colidx;
    if (hipMalloc(&h->scratch, (size_t)nnz * sizeof(float)) != hipSuccess)
        return fail("hipMalloc of the rocsparse_sddmm output scratch failed", kHip);
    RS_CHECK(rocsparse_create_dnmat_descr(&h->A, M, K, K, dummy, h->ab_type, rocsparse_order_row));
    RS_CHECK(rocsparse_create_dnmat_descr(&h->B, K, N, K, dummy, h->ab_type,
                                          rocsparse_order_column));
    RS_CHECK(rocsparse_create_csr_descr(&h->C, M, N, nnz, (void*)d_rowptr, (void*)d_colidx,
                                        h->scratch, rocsparse_indextype_i32,
                                        rocsparse_indextype_i32, rocsparse_index_base_zero,
                                        rocsparse_datatype_f32_r));
    size_t bytes = 0;
    RS_CHECK(rocsparse_sddmm_buffer_size(h->handle, rocsparse_operation_none,
                                         rocsparse_operation_none, &h->alpha, h->A, h->B,
                                         &h->beta, h->C, rocsparse_datatype_f32_r, h->alg, &bytes));
    if (hipMalloc(&h->buffer, bytes ? bytes : 4) != hipSuccess)
        return fail("hipMalloc of the rocsparse_sddmm buffer failed", kHip);
    RS_CHECK(rocsparse_sddmm_preprocess(h->handle, rocsparse_operation_none,
                                        rocsparse_operation_none, &h->alpha, h->A, h->B, &h->beta,
                                        h->C, rocsparse_datatype_f32_r, h->alg, h->buffer));
    return kOk;
}

int bsmr_rocsparse_create(uint32_t M, uint32_t N, uint32_t K, uint32_t nnz,
                          const uint32_t* d_rowptr, const uint32_t* d_colidx, int dtype, int alg,
                          void* stream, bsmr_rocsparse** out) {
    g_err.clear();
    if (!out || !d_rowptr || !d_colidx || M == 0 || N == 0 || K == 0 || nnz == 0 ||
        nnz > 0x7fffffffu)
        return fail("bsmr_rocsparse_create: invalid argument", kInvalid);
    *out = nullptr;
    auto* h = new bsmr_rocsparse;
    switch (dtype) {
        case 0: h->ab_type = rocsparse_datatype_f32_r; break;
        case 1: h->ab_type = rocsparse_datatype_f16_r; break;
        case 2: h->ab_type = rocsparse_datatype_bf16_r; break;
        default: delete h; return fail("bsmr_rocsparse_create: unknown dtype", kUnsupported);
    }
    h->alg = alg == 1 ? rocsparse_sddmm_alg_dense : rocsparse_sddmm_alg_default;
    int rc = create_impl(h, M, N, K, nnz, d_rowptr, d_colidx, stream);
    if (rc != kOk) {
        bsmr_rocsparse_destroy(h);
        return rc;
    }
    *out = h;
    return kOk;
}

int bsmr_rocsparse_sddmm(bsmr_rocsparse* h, const void* dA, const void* dB, float* dP) {
    if (!h || !dA || !dB || !dP) return fail("bsmr_rocsparse_sddmm: invalid argument", kInvalid);
    RS_CHECK(rocsparse_dnmat_set_values(h->A, (void*)dA));
    RS_CHECK(rocsparse_dnmat_set_values(h->B, (void*)dB));
    RS_CHECK(rocsparse_spmat_set_values(h->C, dP));
    RS_CHECK(rocsparse_sddmm(h->handle, rocsparse_operation_none, rocsparse_operation_none,
                             &h->alpha, h->A, h->B, &h->beta, h->C, rocsparse_datatype_f32_r,
                             h->alg, h->buffer));
    return kOk;
}

}  // extern "C"
