// mfma_probe.hip -- calibration of the f32 MFMA ceiling on this MI355X.
//
// Back-to-back v_mfma_f32_32x32x2_f32 on register operands (no LDS, no
// memory in the loop), 4 independent accumulators per wave, waves per SIMD
// 1..3, random or zero operands.  Reports TFLOP/s, the fraction of the
// 157.3 TF spec (2.4 GHz), and the in-kernel clock from s_memtime /
// s_memrealtime (100 MHz), so the predictive kernel's roofline fraction can be
// read against what the matrix pipe sustains under load.
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_probe.hip -o /tmp/mfma_probe && /tmp/mfma_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int W>
__global__ __launch_bounds__(256, W) void probe(const float *in, float *out, int iters, unsigned long long *clk) {
    const int lane = threadIdx.x & 63;
    float a0 = in[lane], a1 = in[64 + lane], a2 = in[128 + lane], a3 = in[192 + lane];
    float b = in[256 + lane];
    f32x16 acc[4];
    for (int i = 0; i < 4; ++i)
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b, acc[0], 0, 0, 0);
            acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b, acc[1], 0, 0, 0);
            acc[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a2, b, acc[2], 0, 0, 0);
            acc[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(a3, b, acc[3], 0, 0, 0);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
    for (int i = 0; i < 4; ++i)
        for (int r = 0; r < 16; ++r) s += acc[i][r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

// The predictive kernel's step mix: 4 MFMAs + one ds_read_b128 (A operands)
// + coordinates from LDS + the K* VALU chain (sub, sub, mul, fma, mul, exp).
// MIX bits: 1 = LDS reads, 2 = K* VALU chain, 4 = exp in the chain,
// 8 = accumulators pinned to AGPRs (inline asm) instead of VGPRs.
template <int W, int MIX>
__global__ __launch_bounds__(256, W) void probe_mix(const float *in, float *out, int iters, unsigned long long *clk) {
    __shared__ __attribute__((aligned(16))) float lds[2 * 64 * 32 * 4 + 3 * 64];
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 2 * 64 * 32 * 4 + 3 * 64; i += 256) lds[i] = in[i & 255];
    __syncthreads();
    const float4 *pa = reinterpret_cast<const float4 *>(lds) + lane;
    const float *pc = lds + 2 * 64 * 32 * 4 + (lane >> 5);
    const float xq = in[lane], yq = in[64 + lane], cexp = -2.9f;
    float4 a = pa[0];
    float b = in[256 + lane], x = in[lane + 1], y = in[lane + 2];
    f32x16 acc[4];
    for (int i = 0; i < 4; ++i)
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int p = 0; p < 32; ++p) {
            float4 an = a;
            float xn = x, yn = y;
            if (MIX & 1) {
                an = pa[((p + 1) & 31) * 64];
                xn = pc[2 * ((p + 1) & 31)];
                yn = pc[64 + 2 * ((p + 1) & 31)];
            }
            float bn = b;
            if (MIX & 2) {
                const float dx = x - xq, dy = y - yq;
                const float d = cexp * fmaf(dy, dy, dx * dx);
                bn = (MIX & 4) ? __builtin_amdgcn_exp2f(d) : d;
            }
            if (MIX & 8) {
                asm volatile("v_mfma_f32_32x32x2_f32 %0, %1, %2, %0" : "+a"(acc[0]) : "v"(a.x), "v"(b));
                asm volatile("v_mfma_f32_32x32x2_f32 %0, %1, %2, %0" : "+a"(acc[1]) : "v"(a.y), "v"(b));
                asm volatile("v_mfma_f32_32x32x2_f32 %0, %1, %2, %0" : "+a"(acc[2]) : "v"(a.z), "v"(b));
                asm volatile("v_mfma_f32_32x32x2_f32 %0, %1, %2, %0" : "+a"(acc[3]) : "v"(a.w), "v"(b));
            } else {
                acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b, acc[0], 0, 0, 0);
                acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b, acc[1], 0, 0, 0);
                acc[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b, acc[2], 0, 0, 0);
                acc[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b, acc[3], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            a = an; b = bn; x = xn; y = yn;
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
    for (int i = 0; i < 4; ++i)
        for (int r = 0; r < 16; ++r) s += acc[i][r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

// R = 8 row blocks per K* value (one wave per SIMD, 512 registers): per step
// two ds_read_b128 (eight A operands), coordinates, the K* chain and 8 MFMAs.
__global__ __launch_bounds__(256, 1) void probe_r8(const float *in, float *out, int iters, unsigned long long *clk) {
    __shared__ __attribute__((aligned(16))) float lds[2 * 64 * 32 * 8 + 3 * 64];
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 2 * 64 * 32 * 8 + 3 * 64; i += 256) lds[i] = in[i & 255];
    __syncthreads();
    const float4 *pa = reinterpret_cast<const float4 *>(lds) + 2 * lane;
    const float *pc = lds + 2 * 64 * 32 * 8 + (lane >> 5);
    const float xq = in[lane], yq = in[64 + lane], cexp = -2.9f;
    float4 a = pa[0], a2 = pa[1];
    float b = in[256 + lane], x = in[lane + 1], y = in[lane + 2];
    f32x16 acc[8];
    for (int i = 0; i < 8; ++i)
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int p = 0; p < 32; ++p) {
            const float4 an = pa[((p + 1) & 31) * 128], a2n = pa[((p + 1) & 31) * 128 + 1];
            const float xn = pc[2 * ((p + 1) & 31)], yn = pc[64 + 2 * ((p + 1) & 31)];
            const float dx = x - xq, dy = y - yq;
            const float bn = __builtin_amdgcn_exp2f(cexp * fmaf(dy, dy, dx * dx));
            acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b, acc[0], 0, 0, 0);
            acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b, acc[1], 0, 0, 0);
            acc[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b, acc[2], 0, 0, 0);
            acc[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b, acc[3], 0, 0, 0);
            acc[4] = __builtin_amdgcn_mfma_f32_32x32x2f32(a2.x, b, acc[4], 0, 0, 0);
            acc[5] = __builtin_amdgcn_mfma_f32_32x32x2f32(a2.y, b, acc[5], 0, 0, 0);
            acc[6] = __builtin_amdgcn_mfma_f32_32x32x2f32(a2.z, b, acc[6], 0, 0, 0);
            acc[7] = __builtin_amdgcn_mfma_f32_32x32x2f32(a2.w, b, acc[7], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            a = an; a2 = a2n; b = bn; x = xn; y = yn;
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
    for (int i = 0; i < 8; ++i)
        for (int r = 0; r < 16; ++r) s += acc[i][r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

// 16x16x4 f32 with 16 row blocks per K* value (256 rows x 16 queries per
// wave, 64 accumulator registers): per step four ds_read_b128, coordinates,
// the K* chain and 16 MFMAs.  W waves per SIMD.
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <int W>
__global__ __launch_bounds__(256, W) void probe_16(const float *in, float *out, int iters, unsigned long long *clk) {
    __shared__ __attribute__((aligned(16))) float lds[4 * 64 * 16 * 4 + 3 * 64];
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 4 * 64 * 16 * 4 + 3 * 64; i += 256) lds[i] = in[i & 255];
    __syncthreads();
    const float4 *pa = reinterpret_cast<const float4 *>(lds) + (lane >> 4) * 16 + (lane & 15);
    const float *pc = lds + 4 * 64 * 16 * 4 + (lane >> 4);
    const float xq = in[lane], yq = in[64 + lane], cexp = -2.9f;
    float4 a[4];
    for (int j = 0; j < 4; ++j) a[j] = pa[j * 1024];
    float b = in[256 + lane], x = in[lane + 1], y = in[lane + 2];
    f32x4 acc[16];
    for (int i = 0; i < 16; ++i)
        for (int r = 0; r < 4; ++r) acc[i][r] = 0.f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int p = 0; p < 16; ++p) {
            float4 an[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) an[j] = pa[j * 1024 + ((p + 1) & 15) * 64];
            const float xn = pc[4 * ((p + 1) & 15)], yn = pc[64 + 4 * ((p + 1) & 15)];
            const float dx = x - xq, dy = y - yq;
            const float bn = __builtin_amdgcn_exp2f(cexp * fmaf(dy, dy, dx * dx));
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                acc[4 * j + 0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j].x, b, acc[4 * j + 0], 0, 0, 0);
                acc[4 * j + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j].y, b, acc[4 * j + 1], 0, 0, 0);
                acc[4 * j + 2] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j].z, b, acc[4 * j + 2], 0, 0, 0);
                acc[4 * j + 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j].w, b, acc[4 * j + 3], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < 4; ++j) a[j] = an[j];
            b = bn; x = xn; y = yn;
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
    for (int i = 0; i < 16; ++i)
        for (int r = 0; r < 4; ++r) s += acc[i][r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

// Wave specialisation: 8 waves per block, two per SIMD.  Waves 0-3 only read
// LDS and issue MFMAs (four 32x32x2 per step, A and B from LDS); waves 4-7 only
// run the K* VALU chain (exp included) and write LDS.  PRODUCER_WORK = K*
// values per producer lane per consumer step x 8 (8 = one per step).
template <int PW>
__global__ __launch_bounds__(512, 1) void probe_spec(const float *in, float *out, int iters, unsigned long long *clk) {
    __shared__ __attribute__((aligned(16))) float lds[2 * 64 * 32 * 4 + 4096];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 2 * 64 * 32 * 4 + 4096; i += 512) lds[i] = in[i & 255];
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
    if (wave < 4) {
        const float4 *pa = reinterpret_cast<const float4 *>(lds) + lane;
        const float *pb = lds + 2 * 64 * 32 * 4 + lane;
        f32x16 acc[4];
        for (int i = 0; i < 4; ++i)
            for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
        float4 a = pa[0];
        float b = pb[0];
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int p = 0; p < 32; ++p) {
                const float4 an = pa[((p + 1) & 31) * 64];
                const float bn = pb[((p + 1) & 31) * 64];
                acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b, acc[0], 0, 0, 0);
                acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b, acc[1], 0, 0, 0);
                acc[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b, acc[2], 0, 0, 0);
                acc[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b, acc[3], 0, 0, 0);
                a = an;
                b = bn;
            }
        }
        for (int i = 0; i < 4; ++i)
            for (int r = 0; r < 16; ++r) s += acc[i][r];
    } else {
        const float xq = in[lane], yq = in[64 + lane], cexp = -2.9f;
        const float *pc = lds + 2 * 64 * 32 * 4 + 2048;
        float *pw = lds + 2 * 64 * 32 * 4 + 2048 + 256 + (wave - 4) * 64 + lane;
        for (int it = 0; it < iters; ++it) {
#pragma unroll 4
            for (int p = 0; p < 32 * PW / 8; ++p) {
                const float dx = pc[p & 63] - xq, dy = pc[64 + (p & 63)] - yq;
                const float v = __builtin_amdgcn_exp2f(cexp * fmaf(dy, dy, dx * dx));
                pw[(p & 3) * 256] = v;
                s += v;
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

#define CHECK(x)                                                                         \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

template <int W, int MIX = -1>
void run(bool zero, int blocks_per_cu) {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int blocks = cus * blocks_per_cu;
    const int iters = MIX < 0 ? 4000 : 500;
    std::vector<float> h(320);
    for (auto &v : h) v = zero ? 0.f : (float)rand() / (float)RAND_MAX - 0.5f;
    float *in, *out;
    unsigned long long *clk;
    CHECK(hipMalloc(&in, 320 * 4));
    CHECK(hipMalloc(&out, (size_t)blocks * 256 * 4));
    CHECK(hipMalloc(&clk, (size_t)blocks * 16));
    CHECK(hipMemcpy(in, h.data(), 320 * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto launch = [&]() {
        if constexpr (MIX >= 100)
            hipLaunchKernelGGL(probe_spec<MIX - 100>, dim3(blocks), dim3(512), 0, 0, in, out, iters, clk);
        else if constexpr (MIX == 98)
            hipLaunchKernelGGL(probe_16<W>, dim3(blocks), dim3(256), 0, 0, in, out, iters, clk);
        else if constexpr (MIX == 99)
            hipLaunchKernelGGL(probe_r8, dim3(blocks), dim3(256), 0, 0, in, out, iters, clk);
        else if constexpr (MIX < 0)
            hipLaunchKernelGGL(probe<W>, dim3(blocks), dim3(256), 0, 0, in, out, iters, clk);
        else
            hipLaunchKernelGGL((probe_mix<W, MIX < 0 ? 0 : MIX>), dim3(blocks), dim3(256), 0, 0, in, out, iters, clk);
    };
    for (int w = 0; w < 20; ++w) launch();
    CHECK(hipEventRecord(e0));
    const int reps = 20;
    for (int w = 0; w < reps; ++w) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> hc((size_t)blocks * 2);
    CHECK(hipMemcpy(hc.data(), clk, hc.size() * 8, hipMemcpyDeviceToHost));
    double ghz = 0;
    for (int b = 0; b < blocks; ++b) ghz += (double)hc[2 * b] / (double)hc[2 * b + 1] * 0.1;
    ghz /= blocks;
    const double flops = (double)reps * blocks * 4 /*waves*/ * iters * (MIX < 0 ? 32 : MIX == 99 ? 256 : MIX == 98 ? 128 : 128) * 4096.0;  // spec: 4 consumer waves x 128
    const double tf = flops / (ms * 1e-3) / 1e12;
    const char *what = "bare MFMA loop (4 x 32x32x2 per step, register operands)";
    if (MIX == 98) what = "16x16x4: 16 MFMAs + 4 ds_read_b128 + K* chain per step (256 rows x 16 q / wave)";
    else if (MIX == 99) what = "32x32x2: 8 MFMAs + 2 ds_read_b128 + K* chain per step (256 rows x 32 q / wave)";
    else if (MIX >= 100) what = "specialised: MFMA-only waves 0-3 beside VALU-only (K* + ds_write) waves 4-7";
    else if (MIX >= 0) {
        static char buf[160];
        snprintf(buf, sizeof buf, "32x32x2, 4 MFMAs per step%s%s%s%s", (MIX & 1) ? " + LDS reads" : "",
                 (MIX & 2) ? " + K* VALU chain" : "", (MIX & 4) ? " with exp" : "", (MIX & 8) ? ", acc in AGPRs" : "");
        what = buf;
    }
    printf("[%s%s] ", what, MIX >= 100 ? (MIX == 100 ? ", producers idle" : MIX == 102 ? ", 1 K* / 4 steps" :
                                           MIX == 108 ? ", 1 K* / step" : ", 2 K* / step") : "");
    if (MIX >= 100) ghz = 2.4;  // per-wave stamps are not a clock here (consumers finish first)
    printf("waves/SIMD %d (launch_bounds %d) %s: %.1f TF (%.1f%% of 157.3)  in-kernel clock %.3f GHz  => %.1f%% of clock-scaled peak\n",
           blocks_per_cu, W, zero ? "zero  " : "random", tf, tf / 157.3 * 100, ghz, tf / (157.3 * ghz / 2.4) * 100);
    CHECK(hipFree(in));
    CHECK(hipFree(out));
    CHECK(hipFree(clk));
}

int main() {
    run<1>(false, 1);
    run<2>(false, 2);
    run<2>(true, 2);
    run<1, 3>(false, 1);
    run<1, 7>(false, 1);
    run<1, 11>(false, 1);
    run<1, 15>(false, 1);
    run<2, 3>(false, 2);
    run<2, 7>(false, 2);
    run<2, 11>(false, 2);
    run<2, 15>(false, 2);
    run<1, 99>(false, 1);
    run<2, 98>(false, 2);
    run<1, 100>(false, 1);
    run<1, 102>(false, 1);
    run<1, 108>(false, 1);
    run<1, 116>(false, 1);
    return 0;
}
