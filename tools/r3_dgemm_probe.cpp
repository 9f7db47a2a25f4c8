// Round-3 probe: rocBLAS dgemm efficiency on the recursive inverse's shapes (top level at N = 16384:
// S[:, p] = B[:, p0:h] Ainv[p0:h, p] panels, m = 8192, panel width w, K = h - p0).
//   hipcc -O2 --offload-arch=gfx950 tools/r3_dgemm_probe.cpp -lrocblas -o tools/r3_dgemm_probe.bin
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <cstdio>

int main() {
    rocblas_handle h;
    rocblas_create_handle(&h);
    const int ld = 16384;
    double *A, *B, *C;
    (void)hipMalloc(&A, sizeof(double) * (size_t)ld * 8192);
    (void)hipMalloc(&B, sizeof(double) * (size_t)ld * 8192);
    (void)hipMalloc(&C, sizeof(double) * (size_t)ld * 8192);
    (void)hipMemset(A, 0x3f, sizeof(double) * (size_t)ld * 8192);
    (void)hipMemset(B, 0x3f, sizeof(double) * (size_t)ld * 8192);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const double one = 1.0, zero = 0.0;
    struct S { int m, n, k; } shapes[] = {
        {8192, 512, 8192}, {8192, 512, 4096}, {8192, 512, 1024}, {8192, 1024, 8192}, {8192, 8192, 8192},
        {16384, 512, 8192},
        // second level (h = 4096): S panels m x w x K, X21 panels w x h x K
        {4096, 512, 4096}, {4096, 512, 3584}, {4096, 512, 2048}, {4096, 512, 1024}, {4096, 512, 512},
        {4096, 256, 4096}, {4096, 384, 4096}, {4096, 640, 4096}, {4096, 768, 4096}, {4096, 1024, 4096},
        {4096, 2048, 4096}, {4096, 4096, 4096}, {512, 4096, 4096}, {512, 4096, 2048}, {1024, 4096, 4096},
        {4096, 512, 4000}, {4096, 528, 4096},
        // third level (h = 2048)
        {2048, 512, 2048}, {2048, 1024, 2048}, {2048, 2048, 2048}, {512, 2048, 2048}, {2048, 256, 2048}};
    for (auto sh : shapes) {
        auto run = [&] {
            rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, sh.m, sh.n, sh.k, &one, A, ld, B, ld, &zero,
                          C, ld);
        };
        for (int r = 0; r < 3; ++r) run();
        (void)hipEventRecord(e0, 0);
        for (int r = 0; r < 10; ++r) run();
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double us = 1e3 * ms / 10, tf = 2.0 * sh.m * sh.n * sh.k / (us * 1e-6) / 1e12;
        printf("dgemm NN m=%5d n=%5d k=%5d: %8.1f us  %5.1f TF  (%.2f of 78.6)\n", sh.m, sh.n, sh.k, us, tf, tf / 78.6);
    }
    return 0;
}
