// Micro-benchmark of the blocked Cholesky's chain kernels in isolation
// (chol_diag_kernel, chol_diag_mfma_kernel, chol_trsm_kernel) at C4's leading dimension, with
// s_memtime phase stamps (-DSBO_CHOL_STAMPS).  GPU diagnostic:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DSBO_CHOL_STAMPS -I/opt/rocm/include \
//         tools/chol_micro.hip -o /tmp/chol_micro && /tmp/chol_micro
#include "../safe_bayesian_optimization_amd/csrc/kernels.hip"

#include <cstdio>
#include <vector>

int main() {
    const int64_t n = 16384, ld = n, kb = 128, m2 = n - kb;
    std::vector<float> h((size_t)kb * ld * 2, 0.0f);
    // an SPD 128 x 128 block (diagonally dominant) and a panel below it
    for (int j = 0; j < kb; ++j)
        for (int64_t i = 0; i < n; ++i) h[i + (size_t)j * ld] = (i == j) ? 200.0f : 0.5f / (1.0f + (float)((i * 7 + j * 3) % 13));
    float *dA = nullptr;
    int *info = nullptr;
    (void)hipMalloc(&dA, sizeof(float) * (size_t)kb * ld);
    (void)hipMalloc(&info, sizeof(int));
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    unsigned long long st[16];
    std::vector<float> out[2], pan[2];
    for (int rep = 0; rep < 6; ++rep) {
        const int ver = rep % 2;   // 0: chol_diag_kernel, 1: chol_diag_mfma_kernel
        (void)hipMemcpy(dA, h.data(), sizeof(float) * (size_t)kb * ld, hipMemcpyHostToDevice);
        (void)hipMemset(info, 0, sizeof(int));
        (void)hipEventRecord(e0, 0);
        (void)sbo::launch_chol_diag(0, dA, ld, (int)kb, 0, info, ver);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms_d = 0.f;
        (void)hipEventElapsedTime(&ms_d, e0, e1);
        (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(sbo::g_chol_stamps), sizeof(st));
        printf("diag v%d: %.1f us  | memtime ticks: load %llu, panels %llu, updates %llu, factor total %llu, store %llu\n",
               ver, ms_d * 1e3, st[1] - st[0], st[4], st[5], st[2] - st[1], st[3] - st[2]);
        out[ver].resize((size_t)kb * kb);
        for (int j = 0; j < kb; ++j)
            (void)hipMemcpy(out[ver].data() + (size_t)j * kb, dA + (size_t)j * ld, sizeof(float) * kb, hipMemcpyDeviceToHost);
        (void)hipEventRecord(e0, 0);
        (void)sbo::launch_chol_trsm(0, dA, ld, (int)kb, dA + kb, m2, ver);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms_t = 0.f;
        (void)hipEventElapsedTime(&ms_t, e0, e1);
        (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(sbo::g_chol_stamps), sizeof(st));
        printf("trsm v%d (m2 %lld): %.1f us | block 0 ticks: load %llu, solve %llu, store %llu\n", ver, (long long)m2,
               ms_t * 1e3, st[9] - st[8], st[10] - st[9], st[11] - st[10]);
        pan[ver].resize((size_t)m2 * kb);
        for (int j = 0; j < kb; ++j)
            (void)hipMemcpy(pan[ver].data() + (size_t)j * m2, dA + kb + (size_t)j * ld, sizeof(float) * m2,
                            hipMemcpyDeviceToHost);
    }
    int hinfo = 0;
    (void)hipMemcpy(&hinfo, info, sizeof(int), hipMemcpyDeviceToHost);
    size_t diff = 0;
    for (int j = 0; j < kb; ++j)
        for (int i = j; i < kb; ++i) diff += out[0][i + (size_t)j * kb] != out[1][i + (size_t)j * kb];
    size_t pdiff = 0;
    for (size_t i = 0; i < pan[0].size(); ++i) pdiff += pan[0][i] != pan[1][i];
    printf("info %d; diagonal block factors v0 vs v1: %zu of %lld lower entries differ; panels: %zu of %zu differ "
           "(s_memtime ticks = shader cycles)\n",
           hinfo, diff, (long long)kb * (kb + 1) / 2, pdiff, pan[0].size());
    return 0;
}
