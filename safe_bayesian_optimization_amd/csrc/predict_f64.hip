// predict_f64.hip -- the precise predictive sweep (a3+a4, SBO_OPT_PRECISION):
// V = A K*^T with A = sf2 L^-1 in f64, K* in f64, f64 MFMA accumulation
// (v_mfma_f64_16x16x4_f64), f64 per-row-block partials and f64 mean.
//
// Why: the default sweep (predict_x3.hip) rounds A to f32 and accumulates in
// f32.  When the posterior variance is small against sf2 -- dense data, e.g.
// N = 16384 on the mapping node's own box [0, 1] x [0, 2.5]
// (config/lpsc.yaml:32-37), sigma^2 ~ 2e-4 .. 3e-3 -- sigma^2 = sf2 - |V|^2
// cancels almost all of |V|^2 ~ 1, and V = A k sums terms far larger than
// itself (|A| |k| >> |A k| for an ill-conditioned K).  Measured there: the
// f32 sweep's variance is 5.0e-4 off the fp64 oracle normwise, an f32 LAPACK
// strtrs on the same factor 6.9e-5; emulated on the host, the rounding of A
// to f32 alone gives 6.6e-5, the f32 accumulation (inside a k-tile's chain
// and across tiles) the rest (tools/r3_stress_accuracy.py).
// With A, K* and every sum in f64 the sweep is exact to f64 rounding times
// the same amplification.
//
// Work items, the tick plan and the persistent walk are those of
// predict_kernel (kernels.hip): workgroup = 256 rows x 128 queries, eight
// waves, wave w owns queries 16w..16w+15 and all 256 rows as sixteen 16-row
// MFMA blocks of f64 accumulators (128 VGPRs).  A stage is half a k-tile
// (32 k x 256 rows x 8 B = 64 KiB + the 32 k's x, y, sf2 alpha in f64),
// double buffered by LDS-DMA, one barrier per stage; inside a stage the A
// operand is stored in MFMA fragment order (pack_f64_kernel), so a lane's A
// operand of one 16x16x4 MFMA is one conflict-free ds_read_b64.
#include <cstdint>

#include "sbo_internal.hpp"

namespace sbo {
namespace {

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int kDH = 32;                       // k per stage (half a k-tile)
constexpr int kDSteps = kDH / 4;              // 16x16x4 MFMA k steps per stage
constexpr int kDRB = kBM / 16;                // 16-row MFMA blocks per wave
constexpr int kDA = kBM * kDH * 8;            // A of a stage: 64 KiB
constexpr int kDC = 3 * kDH * 8;              // x, y, sf2 alpha of the stage's k: 768 B
constexpr int kDSlot = kDA + kDC;
constexpr int kDWaves = kBN / 16;             // 8
constexpr int kDThreads = 64 * kDWaves;
constexpr int kDDescWin = 64;                 // item descriptors (int4) per 1 KiB window
constexpr int kDListWin = 512;                // tile-list entries (u16) per 1 KiB window
constexpr int kDSmem = 2 * kDSlot + 4096;     // two stage slots + two descriptor and two list windows

__device__ __forceinline__ f64x4 mfma_f64(double a, double b, f64x4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// One stage: acc[rb] += A[16 rb + (l & 15)][4 s + (l >> 4)] * K*[4 s + (l >> 4)][q]
// over the stage's eight k steps, and mu += K* sf2 alpha * wmean (1 on the
// last row block, whose items carry the mean; one code path, so the
// accumulators keep their registers).  Software pipeline, pinned with
// scheduling fences: step s issues the LDS reads of step s + 1's sixteen A
// operands and evaluates step s + 1's K* (f64 exp2) beside its own sixteen
// MFMAs, so no MFMA waits on a read or an exp issued in its own step.
__device__ __forceinline__ void stage_steps(const double *__restrict__ pa, const double *__restrict__ pc, double xq,
                                            double yq, double cexp, double wmean, f64x4 (&acc)[kDRB], double &mu) {
    double a[kDRB], an[kDRB];
#pragma unroll
    for (int rb = 0; rb < kDRB; ++rb) a[rb] = pa[rb * 64];
    auto kstar = [&](double xk, double yk) {
        const double dx = xk - xq, dy = yk - yq;
        return exp2(cexp * fma(dy, dy, dx * dx));
    };
    double e = kstar(pc[0], pc[kDH]);
    mu = fma(e, pc[2 * kDH] * wmean, mu);
#pragma unroll
    for (int s = 0; s < kDSteps; ++s) {
        double en = 0.0;
        if (s + 1 < kDSteps) {
            // the next step's coordinates first, then its A operands: the K*
            // below waits only for the coordinates (LDS reads retire in order)
            const double xk = pc[4 * (s + 1)], yk = pc[kDH + 4 * (s + 1)], ak = pc[2 * kDH + 4 * (s + 1)];
#pragma unroll
            for (int rb = 0; rb < kDRB; ++rb) an[rb] = pa[((s + 1) * kDRB + rb) * 64];
            en = kstar(xk, yk);
            mu = fma(en, ak * wmean, mu);
        }
#pragma unroll
        for (int rb = 0; rb < kDRB; ++rb) acc[rb] = mfma_f64(a[rb], e, acc[rb]);
        // one MFMA, then up to two VALU and one LDS read, in turn
#pragma unroll
        for (int j = 0; j < kDRB; ++j) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // VALU
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
        }
        __builtin_amdgcn_sched_barrier(0);
        if (s + 1 < kDSteps) {
#pragma unroll
            for (int rb = 0; rb < kDRB; ++rb) a[rb] = an[rb];
            e = en;
        }
    }
}

__global__ __launch_bounds__(kDThreads, 1) void predict_f64_kernel(
    const double *__restrict__ a64, const double *__restrict__ kc64, const int4 *__restrict__ desc,
    const unsigned short *__restrict__ tl, const int *__restrict__ seg, int P, int n_items, int nI,
    const float *__restrict__ qx, const float *__restrict__ qy, int64_t m, int64_t ldp, double cexp, double m0,
    double *__restrict__ part, double *__restrict__ mean) {
    __shared__ __attribute__((aligned(16))) char smem[kDSmem];
    const int bid = blockIdx.x;
    const int rng = (P % 8 == 0) ? (bid % 8) * (P / 8) + bid / 8 : bid;
    // (bounds are clamped so that a corrupt plan cannot address outside the buffers)
    const int k0 = max(seg[rng], 0), k1 = min(seg[rng + 1], n_items);
    if (k0 >= k1) return;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int r = lane & 15;
    const int g = lane >> 4;
    const int4 *dwin = reinterpret_cast<const int4 *>(smem + 2 * kDSlot);
    const unsigned short *lwin = reinterpret_cast<const unsigned short *>(smem + 2 * kDSlot + 2048);

    // LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave instruction, lane
    // linear), issued from inline asm as in predict_kernel: every wave moves
    // 8 KiB of each 64 KiB A stage, wave 0 also the 768 B of coordinates.
    typedef __attribute__((address_space(3))) char lds_char;
    const uint32_t lds_smem = (uint32_t)(uintptr_t)(lds_char *)(smem);
    const uint32_t lds_wave = lds_smem + (uint32_t)__builtin_amdgcn_readfirstlane(wave) * 1024u;
    const uint32_t lds_dwin = lds_smem + 2u * kDSlot;
    const uint32_t lds_lwin = lds_dwin + 2048u;
    const char *gA = reinterpret_cast<const char *>(a64) + wave * 1024 + lane * 16;
    const char *gC = reinterpret_cast<const char *>(kc64) + lane * 16;
    const char *gD = reinterpret_cast<const char *>(desc) + lane * 16;
    const char *gL = reinterpret_cast<const char *>(tl) + lane * 16;
#define SBO_D_DMA16(gsrc, ldst)                                                                          \
    do {                                                                                                 \
        uint32_t keep_;                                                                                  \
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t" \
                     "s_mov_b32 m0, %0"                                                                  \
                     : "=&s"(keep_)                                                                      \
                     : "v"(gsrc), "s"(ldst)                                                              \
                     : "memory");                                                                        \
    } while (0)
    // stage (packed tile T, half h) into slot buf
#define SBO_D_STAGE(T_, h_, buf)                                                                         \
    do {                                                                                                 \
        const char *s_ = gA + ((int64_t)(T_) * 2 + (h_)) * (int64_t)kDA;                                 \
        const uint32_t d_ = lds_wave + (uint32_t)(buf) * kDSlot;                                         \
        _Pragma("unroll") for (int j_ = 0; j_ < kDA / (1024 * kDWaves); ++j_)                            \
            SBO_D_DMA16(s_ + j_ * kDWaves * 1024, d_ + (uint32_t)(j_ * kDWaves * 1024));                 \
        if (wave == 0 && lane < kDC / 16)                                                                \
            SBO_D_DMA16(gC + ((int64_t)(kt_of_T_) * 2 + (h_)) * kDC, lds_smem + (uint32_t)((buf) * kDSlot + kDA)); \
    } while (0)
#define SBO_D_DESC_WINDOW(w_)                                                                            \
    do {                                                                                                 \
        if (wave == 1) SBO_D_DMA16(gD + (int64_t)(w_) * 1024, lds_dwin + (uint32_t)((w_) & 1) * 1024u);  \
    } while (0)
#define SBO_D_LIST_WINDOW(w_)                                                                            \
    do {                                                                                                 \
        if (wave == 2) SBO_D_DMA16(gL + (int64_t)(w_) * 1024, lds_lwin + (uint32_t)((w_) & 1) * 1024u);  \
    } while (0)
    auto desc_at = [&](int k) {  // wave-uniform descriptor from its (loaded) window
        const int4 d = dwin[((k / kDDescWin) & 1) * kDDescWin + k % kDDescWin];
        const int I = min(max(__builtin_amdgcn_readfirstlane(d.x), 0), nI - 1);
        return make_int4(I, __builtin_amdgcn_readfirstlane(d.y), __builtin_amdgcn_readfirstlane(d.z),
                         __builtin_amdgcn_readfirstlane(d.w));
    };
    auto entry_off = [](const int4 &d) {
        return (uint64_t)(uint32_t)d.z | ((uint64_t)((uint32_t)d.w >> 16) << 32);
    };
    auto list_at = [&](uint64_t e, int I) {  // the k-tile of tile-list entry e (level code ignored: all f64)
        const int t = __builtin_amdgcn_readfirstlane((int)lwin[((e / kDListWin) & 1) * kDListWin + e % kDListWin]) &
                      ((1 << kLevelShift) - 1);
        return min(t, kTilesPerRowBlockStep * (I + 1) - 1);
    };

    // ---- prologue: the first two windows of each kind, the first stage
    SBO_D_DESC_WINDOW(k0 / kDDescWin);
    SBO_D_DESC_WINDOW(k0 / kDDescWin + 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int4 dc = desc_at(k0);
    uint64_t e = entry_off(dc);
    SBO_D_LIST_WINDOW(e / kDListWin);
    SBO_D_LIST_WINDOW(e / kDListWin + 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int t = list_at(e, dc.x);
    {
        const int kt_of_T_ = t;
        SBO_D_STAGE(tile_start(dc.x) + t, 0, 0);
    }
    int64_t q = (int64_t)dc.y * kBN + wave * 16 + r;
    double xq = (double)qx[q < m ? q : m - 1], yq = (double)qy[q < m ? q : m - 1];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    f64x4 acc[kDRB];
#pragma unroll
    for (int rb = 0; rb < kDRB; ++rb) acc[rb] = f64x4{0.0, 0.0, 0.0, 0.0};
    double mu = 0.0;
    int k = k0, j = 0, h = 0, cur = 0;
    for (;;) {
        const int cnt = dc.w & 0xffff;
        // the next stage: the other half of this tile, the next tile of this
        // item, or the first tile of item k + 1
        int kn = k, jn = j, hn = h + 1;
        if (hn == 2) {
            hn = 0;
            jn = j + 1;
            if (jn >= cnt) {
                kn = k + 1;
                jn = 0;
            }
        }
        const bool more = kn < k1;
        int4 dn = dc;
        int tn = t;
        double xqn = xq, yqn = yq;
        if (more) {
            if (kn != k) {
                dn = desc_at(kn);
                if (kn % kDDescWin == 0) SBO_D_DESC_WINDOW(kn / kDDescWin + 1);
                const int64_t qn = (int64_t)dn.y * kBN + wave * 16 + r;
                xqn = (double)qx[qn < m ? qn : m - 1];
                yqn = (double)qy[qn < m ? qn : m - 1];
            }
            if (hn == 0) {
                const uint64_t en = e + 1;
                if (en % kDListWin == 0) SBO_D_LIST_WINDOW(en / kDListWin + 1);
                tn = list_at(en, dn.x);
            }
            const int kt_of_T_ = tn;
            SBO_D_STAGE(tile_start(dn.x) + tn, hn, cur ^ 1);
        }
        const double *pa = reinterpret_cast<const double *>(smem + cur * kDSlot) + lane;
        const double *pc = reinterpret_cast<const double *>(smem + cur * kDSlot + kDA) + g;
        const int I = dc.x;
        stage_steps(pa, pc, xq, yq, cexp, I == nI - 1 ? 1.0 : 0.0, acc, mu);
        if (h == 1 && j == cnt - 1) {
            // item done: column sums of V^2 over its 256 rows; lane l holds
            // rows (l >> 4) + 4 v of every 16-row block, column l & 15
            double sum = 0.0;
#pragma unroll
            for (int rb = 0; rb < kDRB; ++rb) {
#pragma unroll
                for (int c = 0; c < 4; ++c) sum = fma(acc[rb][c], acc[rb][c], sum);
                acc[rb] = f64x4{0.0, 0.0, 0.0, 0.0};
            }
            sum += __shfl_xor(sum, 16);
            sum += __shfl_xor(sum, 32);
            const bool writer = lane < 16 && q < m;
            if (writer) part[(int64_t)I * ldp + q] = sum;
            if (I == nI - 1) {
                mu += __shfl_xor(mu, 16);
                mu += __shfl_xor(mu, 32);
                if (writer) mean[q] = m0 + mu;
                mu = 0.0;
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (!more) break;
        if (kn != k) {
            k = kn;
            dc = dn;
            xq = xqn;
            yq = yqn;
            q = (int64_t)dc.y * kBN + wave * 16 + r;
        }
        if (hn == 0) ++e;
        j = jn;
        h = hn;
        t = tn;
        cur ^= 1;
    }
#undef SBO_D_STAGE
#undef SBO_D_DESC_WINDOW
#undef SBO_D_LIST_WINDOW
#undef SBO_D_DMA16
}

// A = sf2 L^-1 in f64 (from the fit's f64 inverse, lower, column-major, lda
// ld) into packed tiles of row blocks I >= I0: tile (I, t) at
// tile_start(I) + t, two stages of 64 KiB; inside stage h, the A operand of
// MFMA step s (k = 32 h + 4 s + (l >> 4)) and row block rb (row = 16 rb +
// (l & 15)) for lane l at ((s * 16 + rb) * 64 + l).  grid.x = k-tiles of the
// longest row block, grid.y = row block I - I0.
__global__ __launch_bounds__(256) void pack_f64_kernel(const double *__restrict__ Linv, int64_t ld, int64_t n,
                                                       double sf2, int64_t I0, double *__restrict__ a64) {
    const int64_t I = I0 + blockIdx.y;
    const int64_t kb = blockIdx.x;
    if (kb >= (I + 1) * kTilesPerRowBlockStep) return;
    double *tile = a64 + (tile_start(I) + kb) * (int64_t)kTileFloats;
    for (int e = threadIdx.x; e < kTileFloats; e += 256) {
        const int l = e & 63, rb = (e >> 6) & 15, s = (e >> 10) & 7, h = e >> 13;
        const int64_t row = I * kBM + rb * 16 + (l & 15);
        const int64_t col = kb * kBK + h * kDH + s * 4 + (l >> 4);
        tile[e] = (row < n && col < n && col <= row) ? sf2 * Linv[row + col * ld] : 0.0;
    }
}

// Per k-tile and half: x[32], y[32], sf2 alpha[32] in f64 (alpha from the f64
// solve); padding rows: the first point's coordinates, alpha 0.
__global__ void pack_kc64_kernel(const float *__restrict__ x, const float *__restrict__ y,
                                 const double *__restrict__ alpha, int64_t n, int64_t npad, double sf2,
                                 double *__restrict__ kc64) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= npad) return;
    double *c = kc64 + (k / kDH) * (3 * kDH);
    const int o = (int)(k % kDH);
    const bool in = k < n;
    c[o] = (double)(in ? x[k] : x[0]);
    c[kDH + o] = (double)(in ? y[k] : y[0]);
    c[2 * kDH + o] = in ? sf2 * alpha[k] : 0.0;
}

}  // namespace

size_t f64_operand_bytes(int64_t npad) { return 8 * (size_t)total_tiles(npad / kBM) * kTileFloats; }
size_t f64_coord_bytes(int64_t npad) { return 8 * 3 * (size_t)npad; }

hipError_t launch_pack_f64(hipStream_t s, const double *Linv, int64_t ld, int64_t n, int64_t npad, int64_t I0,
                           double sf2, const float *x, const float *y, const double *alpha, double *a64,
                           double *kc64) {
    const int64_t nI = npad / kBM;
    if (I0 < nI) {
        hipLaunchKernelGGL(pack_f64_kernel, dim3((unsigned)(nI * kTilesPerRowBlockStep), (unsigned)(nI - I0)),
                           dim3(256), 0, s, Linv, ld, n, sf2, I0, a64);
    }
    hipLaunchKernelGGL(pack_kc64_kernel, dim3((unsigned)((npad + 255) / 256)), dim3(256), 0, s, x, y, alpha, n, npad,
                       sf2, kc64);
    return hipGetLastError();
}

hipError_t launch_predict_f64(hipStream_t s, const double *a64, const double *kc64, const int4 *desc,
                              const unsigned short *tl, const int *seg, int P, int n_items, int nI, const float *qx,
                              const float *qy, int64_t m, int64_t ldp, double ell, double m0, double *part,
                              double *mean) {
    if (nI <= 0 || m <= 0) return hipSuccess;
    const double cexp = -1.0 / (2.0 * ell * ell * 0.69314718055994530942);
    hipLaunchKernelGGL(predict_f64_kernel, dim3((unsigned)P), dim3(kDThreads), 0, s, a64, kc64, desc, tl, seg, P,
                       n_items, nI, qx, qy, m, ldp, cexp, m0, part, mean);
    return hipGetLastError();
}

}  // namespace sbo
