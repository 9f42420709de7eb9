// rocsparse_cmp.cc -- the rocSPARSE comparator (bench / tests only, not the product).
// Mirrors baseline/base_cusparse/spmm.cu:90-162 of the reference on MI355X:
// CSR int32 A, row-major dense B and C, generic SpMM, warm-up then a timed loop
// with GPU events.  fp32, or fp16 A and B with fp32 C and fp32 compute (rocSPARSE's
// documented mixed-precision SpMM: rocsparse_spmm.h, "f16_r f16_r f32_r f32_r").
#include <hip/hip_runtime.h>
#include <rocsparse/rocsparse.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

static thread_local std::string g_err;

#define RS(x)                                                              \
    do {                                                                   \
        rocsparse_status s_ = (x);                                         \
        if (s_ != rocsparse_status_success) {                              \
            g_err = std::string(#x) + " -> rocsparse status " + std::to_string((int)s_); \
            rc = -1;                                                       \
            goto done;                                                     \
        }                                                                  \
    } while (0)
#define HP(x)                                                              \
    do {                                                                   \
        hipError_t e_ = (x);                                               \
        if (e_ != hipSuccess) {                                            \
            g_err = std::string(#x) + " -> " + hipGetErrorString(e_);      \
            rc = -2;                                                       \
            goto done;                                                     \
        }                                                                  \
    } while (0)

extern "C" {

const char *rs_last_error(void) { return g_err.c_str(); }

// dtype 0: fp32, 1: fp16 A and B (vals/B given as fp32 on the host, converted), fp32 C
// alg: rocsparse_spmm_alg (0 default, 1 csr, 4 csr_row_split, 5 csr_merge/nnz_split, 9 merge_path)
// copies: independent device copies of A and B rotated per call (cold caches)
// out_C (host fp32, M x N) receives the result of the first call; may be null
int rs_spmm_bench(int M, int K, int nnz, const int *row_ptr, const int *col, const float *val, int N, int dtype,
                  int alg, int warmup, int reps, int copies, double *ms_per_call, float *out_C) {
    int rc = 0;
    rocsparse_handle h = nullptr;
    std::vector<rocsparse_spmat_descr> A(copies, nullptr);
    std::vector<rocsparse_dnmat_descr> Bd(copies, nullptr);
    rocsparse_dnmat_descr Cd = nullptr;
    std::vector<void *> bufs;
    void *tmp = nullptr, *dC = nullptr;
    size_t es = dtype == 1 ? 2 : 4;
    rocsparse_datatype dt = dtype == 1 ? rocsparse_datatype_f16_r : rocsparse_datatype_f32_r;
    float alpha = 1.f, beta = 0.f;
    size_t bsz = 0;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    float ms = 0;
    std::vector<uint16_t> v16, b16;
    std::vector<float> b32((size_t)K * N, 0.f);
    for (size_t i = 0; i < b32.size(); i++) b32[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
    if (dtype == 1) {
        v16.resize(nnz);
        b16.resize(b32.size());
        for (int i = 0; i < nnz; i++) { _Float16 x = (_Float16)val[i]; std::memcpy(&v16[i], &x, 2); }
        for (size_t i = 0; i < b32.size(); i++) { _Float16 x = (_Float16)b32[i]; std::memcpy(&b16[i], &x, 2); }
    }
    RS(rocsparse_create_handle(&h));
    HP(hipMalloc(&dC, (size_t)M * N * 4));  // C is fp32 for both dtypes
    for (int c = 0; c < copies; c++) {
        void *drp, *dcol, *dval, *dB;
        HP(hipMalloc(&drp, (size_t)(M + 1) * 4));
        HP(hipMalloc(&dcol, (size_t)nnz * 4 + 4));
        HP(hipMalloc(&dval, (size_t)nnz * es + 4));
        HP(hipMalloc(&dB, (size_t)K * N * es));
        bufs.push_back(drp); bufs.push_back(dcol); bufs.push_back(dval); bufs.push_back(dB);
        HP(hipMemcpy(drp, row_ptr, (size_t)(M + 1) * 4, hipMemcpyHostToDevice));
        HP(hipMemcpy(dcol, col, (size_t)nnz * 4, hipMemcpyHostToDevice));
        HP(hipMemcpy(dval, dtype == 1 ? (const void *)v16.data() : (const void *)val, (size_t)nnz * es, hipMemcpyHostToDevice));
        HP(hipMemcpy(dB, dtype == 1 ? (const void *)b16.data() : (const void *)b32.data(), (size_t)K * N * es, hipMemcpyHostToDevice));
        RS(rocsparse_create_csr_descr(&A[c], M, K, nnz, drp, dcol, dval, rocsparse_indextype_i32, rocsparse_indextype_i32,
                                      rocsparse_index_base_zero, dt));
        RS(rocsparse_create_dnmat_descr(&Bd[c], K, N, N, dB, dt, rocsparse_order_row));
    }
    RS(rocsparse_create_dnmat_descr(&Cd, M, N, N, dC, rocsparse_datatype_f32_r, rocsparse_order_row));
    RS(rocsparse_spmm(h, rocsparse_operation_none, rocsparse_operation_none, &alpha, A[0], Bd[0], &beta, Cd,
                      rocsparse_datatype_f32_r, (rocsparse_spmm_alg)alg, rocsparse_spmm_stage_buffer_size, &bsz, nullptr));
    HP(hipMalloc(&tmp, bsz ? bsz : 4));
    for (int c = 0; c < copies; c++)
        RS(rocsparse_spmm(h, rocsparse_operation_none, rocsparse_operation_none, &alpha, A[c], Bd[c], &beta, Cd,
                          rocsparse_datatype_f32_r, (rocsparse_spmm_alg)alg, rocsparse_spmm_stage_preprocess, &bsz, tmp));
    RS(rocsparse_spmm(h, rocsparse_operation_none, rocsparse_operation_none, &alpha, A[0], Bd[0], &beta, Cd,
                      rocsparse_datatype_f32_r, (rocsparse_spmm_alg)alg, rocsparse_spmm_stage_compute, &bsz, tmp));
    HP(hipDeviceSynchronize());
    if (out_C) HP(hipMemcpy(out_C, dC, (size_t)M * N * 4, hipMemcpyDeviceToHost));
    for (int i = 0; i < warmup; i++)
        RS(rocsparse_spmm(h, rocsparse_operation_none, rocsparse_operation_none, &alpha, A[i % copies], Bd[i % copies],
                          &beta, Cd, rocsparse_datatype_f32_r, (rocsparse_spmm_alg)alg, rocsparse_spmm_stage_compute,
                          &bsz, tmp));
    HP(hipEventCreate(&e0));
    HP(hipEventCreate(&e1));
    HP(hipDeviceSynchronize());
    HP(hipEventRecord(e0, nullptr));
    for (int i = 0; i < reps; i++)
        RS(rocsparse_spmm(h, rocsparse_operation_none, rocsparse_operation_none, &alpha, A[i % copies], Bd[i % copies],
                          &beta, Cd, rocsparse_datatype_f32_r, (rocsparse_spmm_alg)alg, rocsparse_spmm_stage_compute,
                          &bsz, tmp));
    HP(hipEventRecord(e1, nullptr));
    HP(hipEventSynchronize(e1));
    HP(hipEventElapsedTime(&ms, e0, e1));
    *ms_per_call = (double)ms / reps;
done:
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    for (auto a : A) if (a) rocsparse_destroy_spmat_descr(a);
    for (auto b : Bd) if (b) rocsparse_destroy_dnmat_descr(b);
    if (Cd) rocsparse_destroy_dnmat_descr(Cd);
    for (void *p : bufs) (void)hipFree(p);
    if (tmp) (void)hipFree(tmp);
    if (dC) (void)hipFree(dC);
    if (h) rocsparse_destroy_handle(h);
    return rc;
}

}  // extern "C"
