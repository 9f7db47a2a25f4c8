// ozgemm_bench.hip -- A/B of the int8-sliced f64 GEMM (csrc/ozgemm.hip)
// against rocBLAS dgemm on the f64 inverse's own top-level products:
// K = RBF(points) + sn2 I over N points (uniform in a box), L = dpotrf(K),
// Li = dtrtri(L) (rocSOLVER, f64: the reference), h = N / 2, then
//   P1: S = L21 Li11       (L21: N-h x h dense, Li11 lower triangular)
//   P2: X = -Li22 S        (Li22 lower triangular) -- X is Li's lower-left block
// each by dgemm and by the sliced GEMM (ND digits), timed with hip events, and
// the sliced X's error against dtrtri's Li21 (max |dX| / max |Li21| and the
// worst row's |dX|_inf / |Li21 row|_inf), beside dgemm's own.
// Build: make -C safe_bayesian_optimization_amd build/ozgemm.o, then
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I safe_bayesian_optimization_amd/csrc \
//     tools/ozgemm_bench.hip safe_bayesian_optimization_amd/build/ozgemm.o -lrocsolver -lrocblas -o lib/ozgemm_bench
// Usage: lib/ozgemm_bench N xw yw ell nd reps [p2_transposed 1|0]
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "sbo_internal.hpp"

#define CK(x)                                                                        \
    do {                                                                             \
        auto e_ = (x);                                                               \
        if (e_ != 0) {                                                               \
            std::fprintf(stderr, "%s:%d: %s failed (%d)\n", __FILE__, __LINE__, #x, (int)e_); \
            std::exit(1);                                                            \
        }                                                                            \
    } while (0)

__global__ void fill_rbf(const double *x, const double *y, int64_t n, double ell, double sn2, double *K) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, j = blockIdx.y;
    if (i >= n) return;
    const double dx = x[i] - x[j], dy = y[i] - y[j];
    K[i + j * n] = exp(-(dx * dx + dy * dy) / (2.0 * ell * ell)) + (i == j ? sn2 : 0.0);
}
__global__ void zero_upper(double *M, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, j = blockIdx.y;
    if (i < n && i < j) M[i + j * n] = 0.0;
}

int main(int argc, char **argv) {
    const int64_t N = argc > 1 ? std::atoll(argv[1]) : 16384;
    const double xw = argc > 2 ? std::atof(argv[2]) : 1.0, yw = argc > 3 ? std::atof(argv[3]) : 2.5;
    const double ell = argc > 4 ? std::atof(argv[4]) : 0.4;
    const int nd = argc > 5 ? std::atoi(argv[5]) : 6;
    const int reps = argc > 6 ? std::atoi(argv[6]) : 5;
    const int tr = argc > 7 ? std::atoi(argv[7]) : 1;   // P2 in the transposed form (1) or directly (0)
    const int64_t h = N / 2, m = N - h;
    std::vector<double> hx(N), hy(N);
    uint64_t st = 0x9E3779B97F4A7C15ull;
    auto rnd = [&] {
        st ^= st << 13; st ^= st >> 7; st ^= st << 17;
        return (double)(st >> 11) * 0x1.0p-53;
    };
    for (int64_t i = 0; i < N; ++i) {
        hx[i] = xw * rnd();
        hy[i] = yw * rnd();
    }
    // a coarse spatial order (row-major cells of ell) so the factor looks like the fit's
    {
        std::vector<int64_t> p(N);
        for (int64_t i = 0; i < N; ++i) p[i] = i;
        std::sort(p.begin(), p.end(), [&](int64_t a, int64_t b) {
            const long ca = (long)(hy[a] / ell) * 100000 + (long)(hx[a] / ell), cb = (long)(hy[b] / ell) * 100000 + (long)(hx[b] / ell);
            return ca < cb || (ca == cb && a < b);
        });
        std::vector<double> tx(N), ty(N);
        for (int64_t i = 0; i < N; ++i) { tx[i] = hx[p[i]]; ty[i] = hy[p[i]]; }
        hx.swap(tx); hy.swap(ty);
    }
    double *dx, *dy, *L, *Li, *S1, *S2, *X1, *X2;
    CK(hipMalloc(&dx, 8 * N)); CK(hipMalloc(&dy, 8 * N));
    CK(hipMalloc(&L, 8 * N * N)); CK(hipMalloc(&Li, 8 * N * N));
    CK(hipMalloc(&S1, 8 * m * h)); CK(hipMalloc(&S2, 8 * m * h));
    CK(hipMalloc(&X1, 8 * m * h)); CK(hipMalloc(&X2, 8 * m * h));
    CK(hipMemcpy(dx, hx.data(), 8 * N, hipMemcpyHostToDevice));
    CK(hipMemcpy(dy, hy.data(), 8 * N, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(fill_rbf, dim3((unsigned)((N + 255) / 256), (unsigned)N), dim3(256), 0, 0, dx, dy, N, ell, 0.1, L);
    rocblas_handle hb;
    CK(rocblas_create_handle(&hb));
    int *info;
    CK(hipMalloc(&info, 4));
    CK(rocsolver_dpotrf(hb, rocblas_fill_lower, (rocblas_int)N, L, (rocblas_int)N, info));
    hipLaunchKernelGGL(zero_upper, dim3((unsigned)((N + 255) / 256), (unsigned)N), dim3(256), 0, 0, L, N);
    CK(hipMemcpy(Li, L, 8 * N * N, hipMemcpyDeviceToDevice));
    CK(rocsolver_dtrtri(hb, rocblas_fill_lower, rocblas_diagonal_non_unit, (rocblas_int)N, Li, (rocblas_int)N, info));
    CK(hipDeviceSynchronize());
    int hinfo = 0;
    CK(hipMemcpy(&hinfo, info, 4, hipMemcpyDeviceToHost));
    std::printf("N=%lld box %.2f x %.2f ell %.2f nd %d: potrf/trtri info %d\n", (long long)N, xw, yw, ell, nd, hinfo);
    const double one = 1.0, zero = 0.0, mone = -1.0;
    const double *L21 = L + h, *Li11 = Li, *Li22 = Li + h + h * N, *Li21 = Li + h;
    char *ws;
    const size_t wsb = std::max(sbo::gz_workspace_bytes(m, h, h, nd), sbo::gz_workspace_bytes(h, m, m, nd));
    CK(hipMalloc(&ws, wsb));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    float t_d1 = 1e30f, t_d2 = 1e30f, t_z1 = 1e30f, t_z2 = 1e30f;
    for (int r = 0; r < reps; ++r) {
        float t;
        CK(hipEventRecord(e0, 0));
        CK(rocblas_dgemm(hb, rocblas_operation_none, rocblas_operation_none, (rocblas_int)m, (rocblas_int)h, (rocblas_int)h,
                         &one, L21, (rocblas_int)N, Li11, (rocblas_int)N, &zero, S1, (rocblas_int)m));
        CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&t, e0, e1)); t_d1 = std::min(t_d1, t);
        CK(hipEventRecord(e0, 0));
        CK(rocblas_dgemm(hb, rocblas_operation_none, rocblas_operation_none, (rocblas_int)m, (rocblas_int)h, (rocblas_int)m,
                         &mone, Li22, (rocblas_int)N, S1, (rocblas_int)m, &zero, X1, (rocblas_int)m));
        CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&t, e0, e1)); t_d2 = std::min(t_d2, t);
        CK(hipEventRecord(e0, 0));
        CK(sbo::launch_gz_gemm(0, nd, L21, N, Li11, N, m, h, h, 1.0, S2, m, sbo::kGzTriBLower, ws));
        CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&t, e0, e1)); t_z1 = std::min(t_z1, t);
        CK(hipEventRecord(e0, 0));
        if (tr)   // X^T = -S^T Li22^T, stored transposed into X (the library's form)
            CK(sbo::launch_gz_gemm(0, nd, S2, m, Li22, N, h, m, m, -1.0, X2, m,
                                   sbo::kGzTransA | sbo::kGzTransB | sbo::kGzTriBUpper | sbo::kGzTransC, ws));
        else
            CK(sbo::launch_gz_gemm(0, nd, Li22, N, S2, m, m, h, m, -1.0, X2, m, sbo::kGzTriA, ws));
        CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&t, e0, e1)); t_z2 = std::min(t_z2, t);
    }
    // errors against dtrtri's Li21 (host)
    std::vector<double> ref((size_t)(m * h)), a((size_t)(m * h)), b((size_t)(m * h)), s1((size_t)(m * h)), s2((size_t)(m * h));
    CK(hipMemcpy2D(ref.data(), 8 * m, Li21, 8 * N, 8 * m, h, hipMemcpyDeviceToHost));
    CK(hipMemcpy(a.data(), X1, 8 * m * h, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), X2, 8 * m * h, hipMemcpyDeviceToHost));
    CK(hipMemcpy(s1.data(), S1, 8 * m * h, hipMemcpyDeviceToHost));
    CK(hipMemcpy(s2.data(), S2, 8 * m * h, hipMemcpyDeviceToHost));
    auto report = [&](const char *name, const std::vector<double> &got, const std::vector<double> &want) {
        double dmax = 0, vmax = 0, worst_row = 0;
        std::vector<double> rd((size_t)m, 0.0), rv((size_t)m, 0.0);
        for (int64_t j = 0; j < h; ++j)
            for (int64_t i = 0; i < m; ++i) {
                const double d = std::fabs(got[i + j * m] - want[i + j * m]), v = std::fabs(want[i + j * m]);
                dmax = std::max(dmax, d); vmax = std::max(vmax, v);
                rd[i] = std::max(rd[i], d); rv[i] = std::max(rv[i], v);
            }
        for (int64_t i = 0; i < m; ++i) if (rv[i] > 0) worst_row = std::max(worst_row, rd[i] / rv[i]);
        std::printf("  %-28s max|d| %.3e  max|ref| %.3e  rel %.3e  worst row rel %.3e\n", name, dmax, vmax, dmax / vmax, worst_row);
    };
    const double fl1 = (double)m * h * h, fl2 = (double)m * h * m;   // 2 m h K / 2 (triangular)
    std::printf("  P1 S = L21 Li11 (%lld x %lld x %lld, tri B): dgemm %.3f ms (%.1f TF useful), sliced %.3f ms (%.1f TF)\n",
                (long long)m, (long long)h, (long long)h, t_d1, fl1 / t_d1 * 1e-9, t_z1, fl1 / t_z1 * 1e-9);
    std::printf("  P2 X = -Li22 S (%lld x %lld x %lld, %s): dgemm %.3f ms (%.1f TF useful), sliced %.3f ms (%.1f TF)\n",
                (long long)m, (long long)h, (long long)m, tr ? "as X^T = -S^T Li22^T" : "tri A", t_d2, fl2 / t_d2 * 1e-9,
                t_z2, fl2 / t_z2 * 1e-9);
    report("S sliced vs dgemm", s2, s1);
    report("X dgemm vs dtrtri", a, ref);
    report("X sliced vs dtrtri", b, ref);
    return 0;
}
