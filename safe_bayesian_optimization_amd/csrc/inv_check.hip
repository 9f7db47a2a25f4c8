// inv_check.hip -- the fit's run-time accuracy guard of the f64 inverse
// (round 5).
//
// Why: the recursive inverse's top-level products run as an int8-sliced f64
// GEMM (ozgemm.hip, SBO_OPT_INV_OZ) whose error is relative to a row's and a
// column's LARGEST entries, not elementwise.  The precision probe cannot see
// it (its fast and precise sweeps read the same inverse), and the mapper's
// noise and length scale are configuration (config/lpsc.yaml:35-37): a
// smaller noise or a longer length scale raises cond(K) and could eat the
// six-digit margin without a signal.
//
// What: on a guard set of kChkQ queries (a 4 x 4 lattice over the training
// box and 16 training locations) the posterior's V = L^-1 k_q is formed with
// the computed inverse X, V0 = X Kq, and refined once against the f32 factor
// itself, V1 = V0 + X (Kq - L V0), all in f64.  With X = L^-1 (I + E), V1's
// error is O(E^2), so |V1|^2 - |V0|^2 is the inverse's own effect on the
// latent variance sf2 - |V|^2 at those queries (to first order in E), and
// the fit compares its normwise size with the contract (sbo_api.cpp,
// inverse_check).  Cost: three triangular products with 32 right-hand sides
// (two over the f64 inverse, one over the f32 factor) -- one read of each
// lower triangle -- on a stream of their own beside the fit's operand packs.
//
// The mean (round 6): the last right-hand side is not a
// query but the residual r = y - m0 itself, so the same three products give
// z0 = X r and its refinement z1 = z0 + X (r - L z0).  The fit's alpha is
// X^T X r (two f64 dtrmv), so a query's mean is mu0 = m0 + V0^T z0, and the
// exact-inverse mean given the factor m0 + V1^T z1 to O(E^2): their
// difference V0^T dz + dV^T z0 + dV^T dz is the inverse's own share of the
// posterior mean (src/safe_bayesian_optimization_node.cpp:642, mu_), at no
// extra pass over either triangle.
//
// Kernels:
//   chk_kstar_kernel   Kq [rows][Q] (row-major f64) = sf2 exp(-d^2 / 2l^2) for
//                      the kChkQ - 1 queries, r = obs - m0 in the last column
//   chk_trimul_kernel  split-k partial products P[kc][i][c] = sum over k in
//                      chunk kc, k <= i, of T[i + k ld] X[k][c] (T f64 or f32,
//                      lower triangle only: the f32 factor's strictly upper
//                      part holds K's entries), v_mfma_f64_16x16x4_f64,
//                      X staged through LDS 64 k at a time
//   chk_reduce_kernel  Y = sum over the row's chunks (fixed order), or Kq - Y
//   chk_colsum_kernel  per query column: sum dV (2 V0 + dV), sum (V0 + dV)^2,
//                      sum V0 z0 and sum V0 dz + dV z0 + dV dz
#include <cstdint>

#include "sbo_internal.hpp"

namespace sbo {
namespace {

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int kChkWaves = 8;
constexpr int kChkRows = 16 * kChkWaves;  // rows per workgroup: eight waves of 16
constexpr int kChkThreads = 64 * kChkWaves;
constexpr int kChkCB = kChkQ / 16;        // 16-column blocks per wave
constexpr int kChkR = kChkQ - 1;          // the residual's column
constexpr int kChkKC = 1024;              // k per workgroup (split-k chunk)
constexpr int kChkStage = 64;             // k staged in LDS per step
constexpr int kChkLd = kChkQ + 16;        // LDS row stride (doubles): the four
                                          // 16-lane groups of a B read fall on
                                          // two disjoint bank halves

__device__ __forceinline__ f64x4 mfma_f64(double a, double b, f64x4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

__global__ __launch_bounds__(256) void chk_kstar_kernel(const float *__restrict__ x, const float *__restrict__ y,
                                                         const float *__restrict__ obs, double m0, int64_t n,
                                                         int64_t rows, const float *__restrict__ qx,
                                                         const float *__restrict__ qy, double sf2, double inv2l2,
                                                         double *__restrict__ Kq) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= rows * kChkQ) return;
    const int64_t j = idx / kChkQ;
    const int c = (int)(idx % kChkQ);
    double v = 0.0;
    if (j < n) {
        if (c == kChkR) {
            v = (double)obs[j] - m0;   // the residual, as the fit's launch_widen_sub forms it
        } else {
            const double dx = (double)x[j] - (double)qx[c], dy = (double)y[j] - (double)qy[c];
            v = sf2 * exp(-(dx * dx + dy * dy) * inv2l2);
        }
    }
    Kq[idx] = v;
}

// chunks of k a row block's product spans (k < min((rb + 1) 64, n))
__device__ __forceinline__ int chk_chunks(int64_t rb, int64_t n) {
    const int64_t kend = (rb + 1) * kChkRows < n ? (rb + 1) * kChkRows : n;
    return (int)((kend + kChkKC - 1) / kChkKC);
}

// grid (row blocks, chunks); wave w owns rows 16 w .. 16 w + 15 of the row
// block and all kChkQ columns (kChkCB 16 x 16 f64 accumulators).  A fragment
// (lane l): T[row r0 + (l & 15)][k + (l >> 4)], B: X[k + (l >> 4)][16 j + (l & 15)];
// D: row (l >> 4) + 4 v, column l & 15 (cdna_hip_programming.md, f64 MFMA).
// The stage's A fragments are loaded before the X stage is waited for, so
// the triangle's stream (the bound: one read of it) overlaps the staging.
template <class T>
__global__ __launch_bounds__(kChkThreads) void chk_trimul_kernel(const T *__restrict__ Tm, int64_t ld, int64_t n,
                                                                  int64_t rows, const double *__restrict__ X,
                                                                  double *__restrict__ P) {
    __shared__ double xs[kChkStage * kChkLd];
    const int64_t rb = blockIdx.x;
    const int kc = blockIdx.y;
    if (kc >= chk_chunks(rb, n)) return;  // uniform per workgroup
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t r0 = rb * kChkRows + 16 * wave;
    const int64_t row = r0 + (lane & 15);
    const int64_t kb = (int64_t)kc * kChkKC;
    int64_t ke = kb + kChkKC;
    const int64_t rend = (rb + 1) * kChkRows;
    if (ke > rend) ke = rend;
    if (ke > n) ke = n;
    f64x4 acc[kChkCB];
#pragma unroll
    for (int j = 0; j < kChkCB; ++j) acc[j] = f64x4{0.0, 0.0, 0.0, 0.0};
    // software-pipelined (round 6): the next stage's A fragments and X
    // elements are loaded into registers before this stage's MFMAs, so a
    // wave's loads overlap its own arithmetic (the stage-by-stage form waited
    // out a full memory latency per 64 k: ~1.1 ms per f64 product at C4,
    // beside the fit's tail)
    constexpr int kXe = kChkStage * kChkQ / kChkThreads;   // X doubles per thread per stage
    auto load_a = [&](int64_t k0, double (&a)[kChkStage / 4]) {
#pragma unroll
        for (int s = 0; s < kChkStage / 4; ++s) {
            const int64_t k = k0 + 4 * s + (lane >> 4);
            a[s] = (k < ke && k <= row && row < n) ? (double)Tm[row + k * ld] : 0.0;
        }
    };
    auto load_x = [&](int64_t k0, double2 (&xv)[kXe / 2]) {
#pragma unroll
        for (int e = 0; e < kXe; e += 2) {
            const int f = (int)threadIdx.x * 2 + e * kChkThreads;  // element pair index
            const int64_t k = k0 + f / kChkQ;
            xv[e / 2] = k < rows ? *reinterpret_cast<const double2 *>(X + k * kChkQ + f % kChkQ) : double2{0.0, 0.0};
        }
    };
    double a[kChkStage / 4], an[kChkStage / 4];
    double2 xv[kXe / 2];
    load_a(kb, a);
    load_x(kb, xv);
    for (int64_t k0 = kb; k0 < ke; k0 += kChkStage) {
        __syncthreads();   // every wave is done reading the previous stage
        // stage X[k0 .. k0 + 63][0 .. kChkQ - 1] (rows past `rows` read as zero)
#pragma unroll
        for (int e = 0; e < kXe; e += 2) {
            const int f = (int)threadIdx.x * 2 + e * kChkThreads;
            *reinterpret_cast<double2 *>(xs + (f / kChkQ) * kChkLd + f % kChkQ) = xv[e / 2];
        }
        __syncthreads();
        const bool more = k0 + kChkStage < ke;
        if (more) {
            load_a(k0 + kChkStage, an);
            load_x(k0 + kChkStage, xv);
        }
#pragma unroll
        for (int s = 0; s < kChkStage / 4; ++s) {
            const double *xb = xs + (4 * s + (lane >> 4)) * kChkLd + (lane & 15);
#pragma unroll
            for (int j = 0; j < kChkCB; ++j) acc[j] = mfma_f64(a[s], xb[16 * j], acc[j]);
        }
        if (more)
#pragma unroll
            for (int s = 0; s < kChkStage / 4; ++s) a[s] = an[s];
    }
    double *out = P + ((int64_t)kc * rows + r0) * kChkQ;
#pragma unroll
    for (int j = 0; j < kChkCB; ++j)
#pragma unroll
        for (int v = 0; v < 4; ++v) out[((lane >> 4) + 4 * v) * kChkQ + 16 * j + (lane & 15)] = acc[j][v];
}

// Y[i][c] = sum_kc P[kc][i][c] over row i's chunks (ascending), or sub - that
// sum; rows >= n: zero
__global__ __launch_bounds__(256) void chk_reduce_kernel(const double *__restrict__ P, int64_t n, int64_t rows,
                                                          const double *__restrict__ sub, double *__restrict__ Y) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= rows * kChkQ) return;
    const int64_t i = idx / kChkQ;
    double s = 0.0;
    if (i < n) {
        const int nc = chk_chunks(i / kChkRows, n);
        for (int kc = 0; kc < nc; ++kc) s += P[(int64_t)kc * rows * kChkQ + idx];
        if (sub) s = sub[idx] - s;
    }
    Y[idx] = s;
}

// Per query column c (one workgroup each, a fixed-order tree), with z0 =
// V0[:, kChkR] = X r and dz = dV[:, kChkR]:
//   out[4 c]     = sum_i dV (2 V0 + dV)            (|V1|^2 - |V0|^2)
//   out[4 c + 1] = sum_i (V0 + dV)^2               (|V1|^2)
//   out[4 c + 2] = sum_i V0 z0                     (the fit's mean less m0)
//   out[4 c + 3] = sum_i V0 dz + dV z0 + dV dz     (V1^T z1 - V0^T z0)
__global__ __launch_bounds__(256) void chk_colsum_kernel(const double *__restrict__ V0,
                                                          const double *__restrict__ dV, int64_t rows,
                                                          double *__restrict__ out) {
    __shared__ double red[4][256];
    const int c = blockIdx.x;
    double sd = 0.0, sv = 0.0, sm = 0.0, sdm = 0.0;
    for (int64_t i = threadIdx.x; i < rows; i += 256) {
        const double v = V0[i * kChkQ + c], d = dV[i * kChkQ + c];
        const double z = V0[i * kChkQ + kChkR], dz = dV[i * kChkQ + kChkR];
        sd += d * (2.0 * v + d);
        sv += (v + d) * (v + d);
        sm += v * z;
        sdm += v * dz + d * z + d * dz;
    }
    red[0][threadIdx.x] = sd;
    red[1][threadIdx.x] = sv;
    red[2][threadIdx.x] = sm;
    red[3][threadIdx.x] = sdm;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w)
#pragma unroll
            for (int k = 0; k < 4; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x < 4) out[4 * c + threadIdx.x] = red[threadIdx.x][0];
}

template <class T>
hipError_t trimul(hipStream_t s, const T *Tm, int64_t ld, int64_t n, int64_t rows, const double *X, double *P,
                  double *Y, const double *sub) {
    const int64_t nrb = rows / kChkRows;
    const int64_t nkc = (rows + kChkKC - 1) / kChkKC;
    hipLaunchKernelGGL(chk_trimul_kernel<T>, dim3((unsigned)nrb, (unsigned)nkc), dim3(kChkThreads), 0, s, Tm, ld, n,
                       rows, X, P);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int64_t tot = rows * kChkQ;
    hipLaunchKernelGGL(chk_reduce_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, P, n, rows, sub, Y);
    return hipGetLastError();
}

}  // namespace

int64_t inv_check_rows(int64_t n) { return round_up(n, kChkRows); }

size_t inv_check_bytes(int64_t n) {
    const int64_t rows = inv_check_rows(n), nkc = (rows + kChkKC - 1) / kChkKC;
    // Kq, V0, R, dV, the partials, the column sums, the queries
    return sizeof(double) * (size_t)(rows * kChkQ * (4 + nkc) + 4 * kChkQ) + sizeof(float) * 2 * kChkQ;
}

hipError_t launch_inv_check(hipStream_t s, const double *Linv, const float *L, int64_t ld, int64_t n,
                            const float *x, const float *y, const float *obs, double m0, double sf2, double ell,
                            void *work, float **qxy, double **colsums) {
    const int64_t rows = inv_check_rows(n), nkc = (rows + kChkKC - 1) / kChkKC;
    const int64_t blk = rows * kChkQ;
    double *Kq = static_cast<double *>(work), *V0 = Kq + blk, *R = V0 + blk, *dV = R + blk, *P = dV + blk;
    double *cs = P + nkc * blk;
    float *q = reinterpret_cast<float *>(cs + 4 * kChkQ);
    if (qxy) *qxy = q;
    if (colsums) *colsums = cs;
    if (!Linv) return hipSuccess;  // (layout query only)
    hipLaunchKernelGGL(chk_kstar_kernel, dim3((unsigned)((blk + 255) / 256)), dim3(256), 0, s, x, y, obs, m0, n,
                       rows, q, q + kChkQ, sf2, 1.0 / (2.0 * ell * ell), Kq);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = trimul<double>(s, Linv, ld, n, rows, Kq, P, V0, nullptr);   // V0 = X Kq
    if (e == hipSuccess) e = trimul<float>(s, L, ld, n, rows, V0, P, R, Kq);            // R = Kq - L V0
    if (e == hipSuccess) e = trimul<double>(s, Linv, ld, n, rows, R, P, dV, nullptr);    // dV = X R
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(chk_colsum_kernel, dim3(kChkR), dim3(256), 0, s, V0, dV, rows, cs);
    return hipGetLastError();
}

}  // namespace sbo
