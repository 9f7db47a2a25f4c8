// Round-3 probe: the blocked Cholesky's trailing update C -= P P^T (lower, K = 512) and
// the look-ahead block (m x 512, K = 512) by chol_update_kernel against rocBLAS ssyrk /
// sgemm, and the max |difference| of the results.  GPU diagnostic:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I/opt/rocm/include tools/r3_update_probe.hip \
//         -lrocblas -o tools/r3_update_probe.bin
#include "../safe_bayesian_optimization_amd/csrc/kernels.hip"

#include <rocblas/rocblas.h>
#include <cmath>
#include <cstdio>
#include <vector>

int main() {
    const int64_t ld = 16384, K = 512;
    rocblas_handle h;
    rocblas_create_handle(&h);
    std::vector<float> hp((size_t)ld * K);
    for (size_t i = 0; i < hp.size(); ++i) hp[i] = (float)((i * 2654435761u) % 1000003u) / 1000003.0f - 0.5f;
    float *P, *C0, *C1;
    (void)hipMalloc(&P, sizeof(float) * hp.size());
    (void)hipMalloc(&C0, sizeof(float) * (size_t)ld * ld);
    (void)hipMalloc(&C1, sizeof(float) * (size_t)ld * ld);
    (void)hipMemcpy(P, hp.data(), sizeof(float) * hp.size(), hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const float one = 1.0f, m1 = -1.0f;
    auto timeit = [&](auto fn) {
        for (int r = 0; r < 2; ++r) fn();
        (void)hipEventRecord(e0, 0);
        for (int r = 0; r < 5; ++r) fn();
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        return 1e3 * ms / 5;
    };
    for (int64_t m : {16000, 12000, 8000, 4000, 2000}) {
        const double fl = (double)m * m * K;   // syrk flops (lower), m^2 K
        const double t_rb = timeit([&] {
            rocblas_ssyrk(h, rocblas_fill_lower, rocblas_operation_none, (int)m, (int)K, &m1, P, (int)ld, &one, C0, (int)ld);
        });
        const double t_own = timeit([&] { (void)sbo::launch_chol_update(0, P, P, ld, m, m, K, true, C1); });
        const double t_rg = timeit([&] {
            rocblas_sgemm(h, rocblas_operation_none, rocblas_operation_transpose, (int)m, 512, (int)K, &m1, P, (int)ld, P,
                          (int)ld, &one, C0, (int)ld);
        });
        const double t_og = timeit([&] { (void)sbo::launch_chol_update(0, P, P, ld, m, 512, K, false, C1); });
        printf("m=%5lld K=%lld  lower: rocblas ssyrk %8.1f us (%5.1f TF)  own %8.1f us (%5.1f TF) | m x 512: rocblas sgemm %7.1f us (%5.1f TF)  own %7.1f us (%5.1f TF)\n",
               (long long)m, (long long)K, t_rb, fl / t_rb * 1e-6, t_own, fl / t_own * 1e-6, t_rg,
               2.0 * m * 512 * K / t_rg * 1e-6, t_og, 2.0 * m * 512 * K / t_og * 1e-6);
    }
    // agreement on one call from zero
    const int64_t m = 3000;
    (void)hipMemset(C0, 0, sizeof(float) * (size_t)ld * ld);
    (void)hipMemset(C1, 0, sizeof(float) * (size_t)ld * ld);
    rocblas_ssyrk(h, rocblas_fill_lower, rocblas_operation_none, (int)m, (int)K, &m1, P, (int)ld, &one, C0, (int)ld);
    (void)sbo::launch_chol_update(0, P, P, ld, m, m, K, true, C1);
    (void)hipDeviceSynchronize();
    std::vector<float> a((size_t)ld * m), b((size_t)ld * m);
    (void)hipMemcpy(a.data(), C0, sizeof(float) * a.size(), hipMemcpyDeviceToHost);
    (void)hipMemcpy(b.data(), C1, sizeof(float) * b.size(), hipMemcpyDeviceToHost);
    double dmax = 0, amax = 0;
    for (int64_t j = 0; j < m; ++j)
        for (int64_t i = j; i < m; ++i) {
            dmax = std::fmax(dmax, std::fabs((double)a[i + j * ld] - b[i + j * ld]));
            amax = std::fmax(amax, std::fabs((double)a[i + j * ld]));
        }
    printf("m=%lld lower update from zero: max |own - ssyrk| %.3e of max |C| %.3e\n", (long long)m, dmax, amax);
    return 0;
}
