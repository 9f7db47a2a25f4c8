// Round-3 probe: the blocked Cholesky's trailing update C -= P P^T (P: m x 128 f32) by
// rocBLAS ssyrk (the fit's current path), by sgemm on the full square, and by a
// bf16 gemm_ex over the split operand (K' = 6 x 128: the six products of the bf16x3
// split, f32 accumulation) -- whole square and in column panels over the lower triangle.
//   hipcc -O2 --offload-arch=gfx950 tools/r3_gemm_probe.cpp -lrocblas -o tools/r3_gemm_probe.bin
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <cstdio>
#include <vector>
#define CK(x) do { if ((x) != 0) { printf("error %s:%d\n", __FILE__, __LINE__); return 1; } } while (0)

int main() {
    rocblas_handle h;
    CK(rocblas_create_handle(&h));
    const int ld = 16384, kb = 128, kk = 6 * kb;
    float *C, *P;
    void *A2, *B2;
    CK(hipMalloc(&C, sizeof(float) * (size_t)ld * ld));
    CK(hipMalloc(&P, sizeof(float) * (size_t)ld * 512));
    CK(hipMalloc(&A2, 2 * (size_t)ld * kk));
    CK(hipMalloc(&B2, 2 * (size_t)ld * kk));
    CK(hipMemset(C, 0, sizeof(float) * (size_t)ld * ld));
    CK(hipMemset(P, 0x3c, sizeof(float) * (size_t)ld * 512));
    CK(hipMemset(A2, 0x3c, 2 * (size_t)ld * kk));
    CK(hipMemset(B2, 0x3c, 2 * (size_t)ld * kk));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const float one = 1.0f, m1 = -1.0f;
    for (int m : {16000, 12000, 8000, 4000, 2000}) {
        auto timeit = [&](const char *what, auto fn) {
            for (int r = 0; r < 3; ++r) fn();
            (void)hipEventRecord(e0, 0);
            const int R = 10;
            for (int r = 0; r < R; ++r) fn();
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double us = 1e3 * ms / R;
            printf("m=%5d %-44s %8.1f us  %6.1f TF (syrk-equivalent m^2 k)\n", m, what, us,
                   (double)m * m * kb / (us * 1e-6) / 1e12);
        };
        timeit("rocblas_ssyrk lower k=512 (per 128 of k)", [&] {
            rocblas_ssyrk(h, rocblas_fill_lower, rocblas_operation_none, m, 512, &m1, P, ld, &one, C, ld);
        });
        timeit("rocblas_sgemm NT m x 512 x 512 (per 128 of k)", [&] {
            rocblas_sgemm(h, rocblas_operation_none, rocblas_operation_transpose, m, 512, 512, &m1, P, ld, P, ld, &one, C, ld);
        });
        timeit("rocblas_sgemm NT m x 384 x 128", [&] {
            rocblas_sgemm(h, rocblas_operation_none, rocblas_operation_transpose, m, 384, 128, &m1, P, ld, P, ld, &one, C, ld);
        });
        timeit("rocblas_ssyrk lower k=128", [&] {
            rocblas_ssyrk(h, rocblas_fill_lower, rocblas_operation_none, m, kb, &m1, P, ld, &one, C, ld);
        });
        timeit("rocblas_sgemm NT full square k=128", [&] {
            rocblas_sgemm(h, rocblas_operation_none, rocblas_operation_transpose, m, m, kb, &m1, P, ld, P, ld, &one, C, ld);
        });
        timeit("gemm_ex bf16 NT full square k=768", [&] {
            rocblas_gemm_ex(h, rocblas_operation_none, rocblas_operation_transpose, m, m, kk, &m1, A2, rocblas_datatype_bf16_r,
                            ld, B2, rocblas_datatype_bf16_r, ld, &one, C, rocblas_datatype_f32_r, ld, C,
                            rocblas_datatype_f32_r, ld, rocblas_datatype_f32_r, rocblas_gemm_algo_standard, 0, 0);
        });
        for (int np : {4, 8}) {
            char nm[64];
            snprintf(nm, sizeof nm, "gemm_ex bf16 k=768, %d lower panels", np);
            timeit(nm, [&] {
                const int w = (m + np - 1) / np;
                for (int p0 = 0; p0 < m; p0 += w) {
                    const int wp = std::min(w, m - p0);
                    rocblas_gemm_ex(h, rocblas_operation_none, rocblas_operation_transpose, m - p0, wp, kk, &m1,
                                    (char *)A2 + 2 * (size_t)p0, rocblas_datatype_bf16_r, ld, (char *)B2 + 2 * (size_t)p0,
                                    rocblas_datatype_bf16_r, ld, &one, C + p0 + (size_t)p0 * ld, rocblas_datatype_f32_r,
                                    ld, C + p0 + (size_t)p0 * ld, rocblas_datatype_f32_r, ld, rocblas_datatype_f32_r,
                                    rocblas_gemm_algo_standard, 0, 0);
                }
            });
            snprintf(nm, sizeof nm, "sgemm k=128, %d lower panels", np);
            timeit(nm, [&] {
                const int w = (m + np - 1) / np;
                for (int p0 = 0; p0 < m; p0 += w) {
                    const int wp = std::min(w, m - p0);
                    rocblas_sgemm(h, rocblas_operation_none, rocblas_operation_transpose, m - p0, wp, kb, &m1, P + p0, ld,
                                  P + p0, ld, &one, C + p0 + (size_t)p0 * ld, ld);
                }
            });
        }
    }
    return 0;
}
