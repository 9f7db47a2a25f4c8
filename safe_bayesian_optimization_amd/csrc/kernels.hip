// kernels.hip -- CDNA4 (gfx950) kernels of the planning-tick hot path.
//
//   rbf_fill      a1  K = sf2 exp(-|xi-xj|^2 / 2l^2) + sn2 I      (HBM-write bound)
//   pack_operand      A = sf2 L^-1 into [BK][BM] tiles, lower triangle only
//   predict       a3+a4  V = A K*^T on f32 MFMA with K* generated in registers;
//                    per row block: sum_rows V^2 (-> variance), sf2 alpha^T K* (-> mean)
//   acquire       a6+a7+a10  sum partials, sd, ComputeSets in f64, masked argmax
//
// The reference has no device code; the math contract is
// SURVEY.md 7, the acquisition restates
// /root/reference/src/safe_bayesian_optimization_node.cpp:409-416.
//
// Compiled with -ffp-contract=off: every fused multiply-add below is explicit,
// so the f64 acquisition arithmetic is the node's plain IEEE double sequence.
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "sbo_internal.hpp"

namespace sbo {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float fast_exp2(float v) { return __builtin_amdgcn_exp2f(v); }

// ------------------------------------------------------------------ a1 fill
// One workgroup: 1024 rows (4 per lane, one 16-B store) x kFillCols columns.
constexpr int kFillCols = 8;

// K[i + j*ld] = sf2 exp(c |a_i - b_j|^2) (+ sn2 where diag && i == j), i < ma, j < mb.
template <bool VEC>
__global__ __launch_bounds__(256) void rbf_fill_kernel(const float *__restrict__ xa,
                                                       const float *__restrict__ ya, int64_t ma,
                                                       const float *__restrict__ xb,
                                                       const float *__restrict__ yb, int64_t mb,
                                                       int64_t ld, float c, float sf2, float sn2,
                                                       int diag, float *__restrict__ K) {
    const int64_t i0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    const int64_t j0 = (int64_t)blockIdx.y * kFillCols;
    if (i0 >= ma) return;
    const bool full = i0 + 3 < ma;
    float xi[4], yi[4];
    if (VEC && full) {
        const float4 a = *reinterpret_cast<const float4 *>(xa + i0);
        const float4 b = *reinterpret_cast<const float4 *>(ya + i0);
        xi[0] = a.x; xi[1] = a.y; xi[2] = a.z; xi[3] = a.w;
        yi[0] = b.x; yi[1] = b.y; yi[2] = b.z; yi[3] = b.w;
    } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t i = i0 + r < ma ? i0 + r : ma - 1;
            xi[r] = xa[i];
            yi[r] = ya[i];
        }
    }
#pragma unroll
    for (int cc = 0; cc < kFillCols; ++cc) {
        const int64_t j = j0 + cc;
        if (j >= mb) break;
        const float xj = xb[j], yj = yb[j];
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float dx = xi[r] - xj, dy = yi[r] - yj;
            v[r] = sf2 * expf(c * fmaf(dy, dy, dx * dx));
            if (diag && i0 + r == j) v[r] += sn2;
        }
        float *col = K + j * ld;
        if (VEC && full) {
            *reinterpret_cast<float4 *>(col + i0) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (i0 + r < ma) col[i0 + r] = v[r];
        }
    }
}

__global__ void sub_scalar_kernel(const float *__restrict__ in, float v, int64_t n,
                                  float *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[i] - v;
}

// (columns j = blockIdx.y + c gridDim.y: grid.y is capped at kMaxGridY)
__global__ void copy_lower_kernel(const float *__restrict__ src, int64_t lds, int64_t n,
                                  float *__restrict__ dst, int64_t ldd) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    for (int64_t j = blockIdx.y; j < n; j += gridDim.y) dst[i + j * ldd] = i >= j ? src[i + j * lds] : 0.0f;
}

// ------------------------------------------------------------ operand pack
// grid.x = k-tiles of the longest row block, grid.y = row block I.
template <class T>
__global__ __launch_bounds__(256) void pack_operand_kernel(const T *__restrict__ Linv,
                                                           int64_t ld, int64_t n, T sf2, int64_t I0,
                                                           float *__restrict__ aug) {
    const int64_t I = I0 + blockIdx.y;
    const int64_t kb = blockIdx.x;
    if (kb >= (I + 1) * kTilesPerRowBlockStep) return;
    float *tile = aug + (tile_start(I) + kb) * kTileFloats;
    // (unrolled: 16 independent loads in flight per thread -- the kernel is a
    // pure stream, 1 GiB of f64 in, 0.5 GiB of f32 out at C4)
#pragma unroll 16
    for (int e = threadIdx.x; e < kTileFloats; e += 256) {
        // inverse of tile_offset: e = ((jj*BK + k)*16 + r)*4 + j3, row = 64 jj + 16 j3 + r
        const int j3 = e & 3, r16 = (e >> 2) & 15, k = (e >> 6) & (kBK - 1), jj = e >> 12;
        const int r = jj * 64 + j3 * 16 + r16;
        const int64_t row = I * kBM + r, col = kb * kBK + k;
        float v = 0.0f;
        if (row < n && col < n && col <= row) v = (float)(sf2 * Linv[row + col * ld]);
        tile[e] = v;
    }
}

// dst[i + j*ldd] = src[i + j*lds] (f32 -> f64), i < m, j < n; lower: zero above the diagonal.
// out[r] = sum_c A[r + c * ld] x[c], c < n, for a few rows r of a column-major
// f64 matrix (one workgroup per row; strided lanes, then a fixed-order tree:
// deterministic) -- rocBLAS dgemv ran a 1 x 16384 strided row in ~300 us
__global__ __launch_bounds__(256) void row_dot_kernel(const double *__restrict__ A, int64_t ld, int64_t n,
                                                      const double *__restrict__ x, double *__restrict__ out) {
    __shared__ double red[256];
    const int64_t r = blockIdx.x;
    double s = 0.0;
    for (int64_t c = threadIdx.x; c < n; c += 256) s = fma(A[r + c * ld], x[c], s);
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o >= 1; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[r] = red[0];
}

// alpha = K^-1 r = X^T (X r) from the fit's f64 inverse X (lower, column-major,
// lda ld, its strictly upper part zero), r = obs - m0 (round 6; was two
// rocBLAS dtrmv: 0.93 + 0.48 ms at C4 for two passes over a 1 GiB triangle).
// Pass 1, z = X r: workgroup (row block of kAlRows rows, k chunk of kAlK
// columns), each thread two consecutive rows (one 16-B load per k: a wave
// reads 1 KiB of a column), r's chunk in LDS; the partial sums of chunk kc go
// to P[kc][row] and alpha_z_reduce_kernel adds them in chunk order.  Pass 2,
// alpha_k = sum_{i >= k} X[i][k] z_i: one wave per column (a contiguous read
// of rows k .. n-1), a fixed-order shuffle tree.  Both deterministic.
constexpr int kAlRows = 512, kAlK = 512;
__global__ __launch_bounds__(256) void alpha_z_kernel(const double *__restrict__ X, int64_t ld, int64_t n,
                                                      const float *__restrict__ obs, double m0,
                                                      double *__restrict__ P) {
    __shared__ double rs[kAlK];
    const int64_t r0 = (int64_t)blockIdx.x * kAlRows, k0 = (int64_t)blockIdx.y * kAlK;
    if (k0 >= r0 + kAlRows || k0 >= n) return;                       // above the diagonal: nothing
    for (int j = threadIdx.x; j < kAlK; j += 256) rs[j] = k0 + j < n ? (double)obs[k0 + j] - m0 : 0.0;
    __syncthreads();
    const int64_t row = r0 + 2 * (int64_t)threadIdx.x;
    const int64_t kend = min(min(k0 + kAlK, n), row + 2);             // k <= row + 1 (the pair's last row)
    double s0 = 0.0, s1 = 0.0;
    if (row < n) {
        const double *col = X + row;
        // (X's strictly upper part is zero: X[row][row + 1] adds nothing).  A
        // 16-B load per k when every (row, k) pair is 16-B aligned (ld even),
        // else two 8-B loads
        if (row + 1 < n && (ld & 1) == 0) {
#pragma unroll 8
            for (int64_t k = k0; k < kend; ++k) {
                const double2 v = *reinterpret_cast<const double2 *>(col + k * ld);
                s0 = fma(v.x, rs[k - k0], s0);
                s1 = fma(v.y, rs[k - k0], s1);
            }
        } else {
            const bool two = row + 1 < n;
#pragma unroll 8
            for (int64_t k = k0; k < kend; ++k) {
                s0 = fma(col[k * ld], rs[k - k0], s0);
                if (two) s1 = fma(col[k * ld + 1], rs[k - k0], s1);
            }
        }
    }
    const int64_t kc = blockIdx.y;
    if (row < n) P[kc * n + row] = s0;
    if (row + 1 < n) P[kc * n + row + 1] = s1;
}
__global__ __launch_bounds__(256) void alpha_z_reduce_kernel(const double *__restrict__ P, int64_t n,
                                                             double *__restrict__ z) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int64_t nkc = i / kAlK + 1;                                 // chunks at or left of the diagonal
    double s = 0.0;
    for (int64_t kc = 0; kc < nkc; ++kc) s += P[kc * n + i];
    z[i] = s;
}
__global__ __launch_bounds__(256) void alpha_xtz_kernel(const double *__restrict__ X, int64_t ld, int64_t n,
                                                        const double *__restrict__ z, double *__restrict__ alpha) {
    const int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (k >= n) return;
    const int lane = threadIdx.x & 63;
    const double *col = X + k * ld;
    double s = 0.0;
    // rows k .. n-1; lane l takes rows i = k + l, k + l + 64, ... (coalesced)
#pragma unroll 4
    for (int64_t i = k + lane; i < n; i += 64) s = fma(col[i], z[i], s);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) alpha[k] = s;
}

// out[i + j * ldo] = (float)d[i + j * ldd] (i < m, j = blockIdx.y)
__global__ void narrow_2d_kernel(const double *__restrict__ d, int64_t ldd, int64_t m, int64_t n,
                                 float *__restrict__ out, int64_t ldo) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    for (int64_t j = blockIdx.y; j < n; j += gridDim.y) out[i + j * ldo] = (float)d[i + j * ldd];
}

// out[j * stride] = (float)d[j]: a row of the f32 factor from an f64 vector
__global__ void narrow_strided_kernel(const double *__restrict__ d, int64_t n, float *__restrict__ out,
                                      int64_t stride) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) out[j * stride] = (float)d[j];
}

__global__ void widen_kernel(const float *__restrict__ src, int64_t lds, int64_t m, int64_t n, int lower,
                             double *__restrict__ dst, int64_t ldd) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    for (int64_t j = blockIdx.y; j < n; j += gridDim.y)
        dst[i + j * ldd] = (!lower || i >= j) ? (double)src[i + j * lds] : 0.0;
}

// Per k-tile coordinates, step-major per lane group: k = 4p + g is stored at
// g*16 + p (x, then y, then sf2*alpha), so lane group g reads the values of
// consecutive k steps p, p+1 as one 8-byte pair.
__device__ __forceinline__ int kcoord_slot(int o) { return (o & 3) * 16 + (o >> 2); }

__global__ void pack_kcoord_kernel(const float *__restrict__ x, const float *__restrict__ y,
                                   const float *__restrict__ alpha, int64_t n, int64_t npad,
                                   float sf2, float *__restrict__ kcoord) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= npad) return;
    const int64_t t = k / kBK;
    const int o = kcoord_slot((int)(k % kBK));
    float *c = kcoord + t * (3 * kBK);
    const bool in = k < n;
    c[o] = in ? x[k] : x[0];
    c[kBK + o] = in ? y[k] : y[0];
    c[2 * kBK + o] = in ? sf2 * alpha[k] : 0.0f;
}

// ---- blocked Cholesky (a2), the factorization step rocSOLVER's spotrf
// spends most of its time in (unblocked potf2 panels, one small workgroup
// each): the kb x kb diagonal block of step k0, in LDS, right-looking in
// panels of kCholPanel columns.  A panel is factored by wave 0 alone in
// registers (lane l holds rows jb + l and jb + 64 + l of the panel; the pivot
// row's values come from their lane by v_readlane, no barrier per column);
// the trailing lower triangle then takes the panel's rank-kCholPanel update
// from all four waves in 4 x 4 element tiles.  Every element sees the same
// fmaf sequence as the column-by-column algorithm (column j ascending,
// fmaf(-L[i][j], L[l][j], a)), so the factor is bitwise that of a plain
// right-looking Cholesky of the block.  f32 as spotrf, correctly rounded sqrt
// and division.  A pivot that is not > 0 (or NaN) stops the factorization:
// info = k0 + j + 1 (the leading minor, rocSOLVER's convention); later blocks
// see info != 0 and leave their data alone.  Column-major, lda = ld; only
// i >= j is written.
constexpr int kCholPanel = 8;
#ifdef SBO_CHOL_STAMPS
// tools/chol_micro.hip only: s_memtime phase stamps of the fit's chain kernels
__device__ unsigned long long g_chol_stamps[16];
#define SBO_CSTAMP(i) do { if (threadIdx.x == 0 && blockIdx.x == 0) g_chol_stamps[i] = __builtin_amdgcn_s_memtime(); } while (0)
#define SBO_CSTAMP_ADD(i, t0) do { if (threadIdx.x == 0 && blockIdx.x == 0) g_chol_stamps[i] += __builtin_amdgcn_s_memtime() - (t0); } while (0)
#else
#define SBO_CSTAMP(i) do { } while (0)
#define SBO_CSTAMP_ADD(i, t0) do { } while (0)
#endif
__device__ __forceinline__ float lane_value(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__global__ __launch_bounds__(256) void chol_diag_kernel(float *__restrict__ A, int64_t ld, int kb, int64_t k0,
                                                        int *__restrict__ info) {
    static_assert(kCholNB <= 128, "two panel rows per lane of wave 0");
    // row stride 132: a row's 8 panel columns are two aligned float4 reads
    __shared__ __attribute__((aligned(16))) float a[kCholNB][kCholNB + 4];
    __shared__ int s_bad;
    if (*info != 0) return;
    SBO_CSTAMP(0);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // the block in, kCholLoad independent loads per thread in flight at a time
    // (one at a time, the reads' latency was most of this kernel)
    constexpr int kCholLoad = 16;
    for (int e0 = 0; e0 < kb * kb; e0 += 256 * kCholLoad) {
        float v[kCholLoad];
#pragma unroll
        for (int u = 0; u < kCholLoad; ++u) {
            const int e = e0 + u * 256 + tid;
            const int i = e % kb, j = e / kb;
            v[u] = (e < kb * kb && i >= j) ? A[i + (int64_t)j * ld] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < kCholLoad; ++u) {
            const int e = e0 + u * 256 + tid;
            const int i = e % kb, j = e / kb;
            if (e < kb * kb && i >= j) a[i][j] = v[u];
        }
    }
    if (tid == 0) s_bad = 0;
    __syncthreads();
    SBO_CSTAMP(1);
#ifdef SBO_CHOL_STAMPS
    if (threadIdx.x == 0) { g_chol_stamps[4] = 0; g_chol_stamps[5] = 0; }
#endif
    for (int jb = 0; jb < kb; jb += kCholPanel) {
        const int w = min(kCholPanel, kb - jb);
#ifdef SBO_CHOL_STAMPS
        const unsigned long long tp0 = __builtin_amdgcn_s_memtime();
#endif
        if (wave == 0) {
            const int r0 = jb + lane, r1 = jb + 64 + lane;
            float p0[kCholPanel], p1[kCholPanel];
#pragma unroll
            for (int c = 0; c < kCholPanel; ++c) {
                p0[c] = (r0 < kb && c < w) ? a[r0][jb + c] : 0.0f;
                p1[c] = (r1 < kb && c < w) ? a[r1][jb + c] : 0.0f;
            }
            int bad = 0;
#pragma unroll
            for (int c = 0; c < kCholPanel; ++c) {
                if (c >= w || bad) continue;   // uniform
                const int j = jb + c;
                const float djj = lane_value(p0[c], c);   // row j is lane c's first row
                // a pivot below FLT_MIN (denormal, flushed or zero) is not
                // positive definite either: its v_rsq_f32 may overflow
                if (!(djj >= 1.17549435e-38f) || !(djj < __builtin_huge_valf())) {
                    bad = j + 1;
                    continue;
                }
                // 1/sqrt(djj) once (v_rsq_f32), the column scaled by it and
                // the pivot as djj * (1/sqrt(djj)): one transcendental on the
                // serial chain instead of a sqrt and two divisions
                const float rs = __builtin_amdgcn_rsqf(djj);
                if (r0 > j) p0[c] = p0[c] * rs;
                else if (r0 == j) p0[c] = djj * rs;
                p1[c] = p1[c] * rs;   // r1 > j always
#pragma unroll
                for (int c2 = c + 1; c2 < kCholPanel; ++c2) {
                    if (c2 >= w) continue;
                    const float lc2 = lane_value(p0[c], c2);   // L[jb + c2][j], lane c2's (already scaled)
                    if (r0 >= jb + c2) p0[c2] = fmaf(-p0[c], lc2, p0[c2]);
                    p1[c2] = fmaf(-p1[c], lc2, p1[c2]);
                }
            }
#pragma unroll
            for (int c = 0; c < kCholPanel; ++c) {
                if (c < w && r0 < kb && r0 >= jb + c) a[r0][jb + c] = p0[c];
                if (c < w && r1 < kb) a[r1][jb + c] = p1[c];
            }
            if (lane == 0 && bad) s_bad = bad;
        }
        __syncthreads();
        SBO_CSTAMP_ADD(4, tp0);
        if (s_bad) break;
#ifdef SBO_CHOL_STAMPS
        const unsigned long long tu0 = __builtin_amdgcn_s_memtime();
#endif
        // rank-w update of the trailing lower triangle [t0, kb) in 4 x 4 tiles
        const int t0 = jb + w, n2 = kb - t0;
        const int nt = (n2 + 3) >> 2, ntiles = nt * (nt + 1) / 2;
        for (int q = tid; q < ntiles; q += 256) {
            int ti = (int)((sqrtf(8.0f * (float)q + 1.0f) - 1.0f) * 0.5f);
            while ((ti + 1) * (ti + 2) / 2 <= q) ++ti;
            while (ti * (ti + 1) / 2 > q) --ti;
            const int tl = q - ti * (ti + 1) / 2;
            const int i0 = t0 + 4 * ti, l0 = t0 + 4 * tl;
            float li[4][kCholPanel], ll[4][kCholPanel];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                // rows past kb read (finite) padding rows of the array; columns
                // past w are masked below
                const float4 *pi = reinterpret_cast<const float4 *>(&a[min(i0 + r, kCholNB - 1)][jb]);
                const float4 *pl = reinterpret_cast<const float4 *>(&a[min(l0 + r, kCholNB - 1)][jb]);
                const float4 i0v = pi[0], i1v = pi[1], l0v = pl[0], l1v = pl[1];
                const float iv[8] = {i0v.x, i0v.y, i0v.z, i0v.w, i1v.x, i1v.y, i1v.z, i1v.w};
                const float lv[8] = {l0v.x, l0v.y, l0v.z, l0v.w, l1v.x, l1v.y, l1v.z, l1v.w};
#pragma unroll
                for (int c = 0; c < kCholPanel; ++c) {
                    li[r][c] = (i0 + r < kb && c < w) ? iv[c] : 0.0f;
                    ll[r][c] = (l0 + r < kb && c < w) ? lv[c] : 0.0f;
                }
            }
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int i = i0 + r, l = l0 + u;
                    if (i < kb && l <= i) {
                        float v = a[i][l];
#pragma unroll
                        for (int c = 0; c < kCholPanel; ++c)
                            if (c < w) v = fmaf(-li[r][c], ll[u][c], v);
                        a[i][l] = v;
                    }
                }
        }
        __syncthreads();
        SBO_CSTAMP_ADD(5, tu0);
    }
    SBO_CSTAMP(2);
    if (s_bad) {
        if (tid == 0) atomicCAS(info, 0, (int)(k0 + s_bad));
        return;
    }
    for (int e = tid; e < kb * kb; e += 256) {
        const int i = e % kb, j = e / kb;
        if (i >= j) A[i + (int64_t)j * ld] = a[i][j];
    }
    SBO_CSTAMP(3);
}

// The same diagonal block in 16-column panels with the trailing updates on
// the matrix cores (chol_diag_kernel's default replacement).  The block is
// padded to 128 x 128 with the identity (pivots 1, zero coupling: the real
// part sees exactly the arithmetic of the kb x kb factorization).  Panel:
// wave 0 in registers, as above (16 columns).  Trailing update: the lower
// triangle of 16 x 16 blocks behind the panel, spread over the four waves,
// each block C -= L_i L_l^T as four v_mfma_f32_16x16x4_f32 over the panel's
// 16 columns -- an MFMA is bit for bit a k-ordered fmaf chain
// (cdna_hip_programming.md section 3), so every element still sees
// fmaf(-L[i][j], L[l][j], a) with j ascending and the factor is bitwise that
// of chol_diag_kernel.  The block in: all 64 loads per thread in flight;
// out: 64 stores per thread issued back to back.
constexpr int kCholPW = 16;
typedef float f32x4_t __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void chol_diag_mfma_kernel(float *__restrict__ A, int64_t ld, int kb, int64_t k0,
                                                             int *__restrict__ info) {
    static_assert(kCholNB == 128, "two panel rows per lane of wave 0, 8 x 16 blocks");
    __shared__ __attribute__((aligned(16))) float a[kCholNB][kCholNB + 4];
    __shared__ int s_bad;
    if (*info != 0) return;
    SBO_CSTAMP(0);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // thread (i, h): row i = tid & 127 of columns h, h + 2, h + 4, ... (coalesced
    // over i), 16 loads in flight per batch
    // (every load unconditional, from inside the kb x kb block: the rows and
    // columns past kb read its last row / column and are replaced after)
    const int li = tid & (kCholNB - 1), lh = tid >> 7;
    const float *colp = A + min(li, kb - 1);
    for (int j0 = 0; j0 < kCholNB; j0 += 32) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = colp[(int64_t)min(j0 + 2 * u + lh, kb - 1) * ld];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int j = j0 + 2 * u + lh;
            a[li][j] = (li < kb && j < kb && li >= j) ? v[u] : (li == j ? 1.0f : 0.0f);
        }
    }
    if (tid == 0) s_bad = 0;
    __syncthreads();
    SBO_CSTAMP(1);
#ifdef SBO_CHOL_STAMPS
    if (threadIdx.x == 0) { g_chol_stamps[4] = 0; g_chol_stamps[5] = 0; }
#endif
    for (int jb = 0; jb < kCholNB; jb += kCholPW) {
#ifdef SBO_CHOL_STAMPS
        const unsigned long long tp0 = __builtin_amdgcn_s_memtime();
#endif
        if (wave == 0) {
            const int r0 = jb + lane, r1 = jb + 64 + lane;
            const int q0 = min(r0, kCholNB - 1), q1 = min(r1, kCholNB - 1);
            float p0[kCholPW], p1[kCholPW];
#pragma unroll
            for (int c4 = 0; c4 < kCholPW / 4; ++c4) {
                const float4 u0 = reinterpret_cast<const float4 *>(&a[q0][jb])[c4];
                const float4 u1 = reinterpret_cast<const float4 *>(&a[q1][jb])[c4];
                p0[4 * c4] = u0.x; p0[4 * c4 + 1] = u0.y; p0[4 * c4 + 2] = u0.z; p0[4 * c4 + 3] = u0.w;
                p1[4 * c4] = u1.x; p1[4 * c4 + 1] = u1.y; p1[4 * c4 + 2] = u1.z; p1[4 * c4 + 3] = u1.w;
            }
            int bad = 0;
#pragma unroll
            for (int c = 0; c < kCholPW; ++c) {
                // (no early exit inside the unrolled panel: a failed pivot is
                // recorded and the rest of the panel computes garbage that the
                // block never stores)
                const int j = jb + c;
                const float djj = lane_value(p0[c], c);   // row j is lane c's first row
                // (pivots below FLT_MIN fail too: v_rsq_f32 of a denormal may overflow)
                if (bad == 0 && (!(djj >= 1.17549435e-38f) || !(djj < __builtin_huge_valf()))) bad = j + 1;
                // every lane, no row tests: the lanes above the diagonal
                // (row < column) compute values of the upper triangle that
                // nothing reads (the lane-mask per column and row would be
                // 136 live SGPR pairs); the diagonal lane's p0[c] is djj, so
                // L_jj = djj * rs there
                const float rs = __builtin_amdgcn_rsqf(djj);
                p0[c] = p0[c] * rs;
                p1[c] = p1[c] * rs;
#pragma unroll
                for (int c2 = c + 1; c2 < kCholPW; ++c2) {
                    const float lc2 = lane_value(p0[c], c2);   // L[jb + c2][j], lane c2's (already scaled)
                    p0[c2] = fmaf(-p0[c], lc2, p0[c2]);
                    p1[c2] = fmaf(-p1[c], lc2, p1[c2]);
                }
            }
            if (r0 < kCholNB) {
#pragma unroll
                for (int c = 0; c < kCholPW; ++c) a[r0][jb + c] = p0[c];
            }
            if (r1 < kCholNB) {
#pragma unroll
                for (int c = 0; c < kCholPW; ++c) a[r1][jb + c] = p1[c];
            }
            if (lane == 0 && bad) s_bad = bad;
        }
        __syncthreads();
        SBO_CSTAMP_ADD(4, tp0);
        if (s_bad) break;
#ifdef SBO_CHOL_STAMPS
        const unsigned long long tu0 = __builtin_amdgcn_s_memtime();
#endif
        // rank-16 update of the trailing lower triangle, 16 x 16 blocks
        const int t0 = jb + kCholPW, nbt = (kCholNB - t0) / 16, nblk = nbt * (nbt + 1) / 2;
        const int fi = lane & 15, fk = lane >> 4;   // operand lane map: A[fi][fk], B[fk][fi]; C row 4 fk + v, col fi
        for (int q = wave; q < nblk; q += 4) {
            int bi = 0, r = q;
            while (r > bi) { r -= bi + 1; ++bi; }
            const int i0 = t0 + 16 * bi, l0 = t0 + 16 * r;
            f32x4_t acc;
#pragma unroll
            for (int v = 0; v < 4; ++v) acc[v] = a[i0 + 4 * fk + v][l0 + fi];
#pragma unroll
            for (int kk = 0; kk < kCholPW / 4; ++kk) {
                const float av = -a[i0 + fi][jb + 4 * kk + fk];
                const float bv = a[l0 + fi][jb + 4 * kk + fk];
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
            }
#pragma unroll
            for (int v = 0; v < 4; ++v) a[i0 + 4 * fk + v][l0 + fi] = acc[v];
        }
        __syncthreads();
        SBO_CSTAMP_ADD(5, tu0);
    }
    SBO_CSTAMP(2);
    if (s_bad) {
        if (tid == 0) atomicCAS(info, 0, (int)(k0 + s_bad));
        return;
    }
    float *colw = A + li + (int64_t)lh * ld;
    for (int j0 = 0; j0 < kCholNB; j0 += 32) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = a[li][j0 + 2 * u + lh];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int j = j0 + 2 * u + lh;
            if (li < kb && j < kb && li >= j) colw[(int64_t)(j0 + 2 * u) * ld] = v[u];
        }
    }
    SBO_CSTAMP(3);
}

// The same diagonal block, left-looking (round 5; SBO_OPT_CHOL_DIAG 1, the
// default -- 2 keeps the right-looking chol_diag_mfma_kernel): before wave 0
// factors a 16-column panel, the four waves bring the panel's columns up to
// date with every factored column in one MFMA chain per 16 x 16 block, the
// accumulator in registers -- each element sees fmaf(-L[i][j], L[l][j], a)
// for j ascending as in the right-looking kernel's per-panel updates, so the
// factor is bitwise the same -- instead of updating the whole trailing
// triangle through LDS after every panel; and the panel itself on all four
// waves (one row per lane) instead of wave 0 (two).
__global__ __launch_bounds__(256) void chol_diag_ll_kernel(float *__restrict__ A, int64_t ld, int kb, int64_t k0,
                                                           int *__restrict__ info) {
    static_assert(kCholNB == 128, "two panel rows per lane of wave 0, 8 x 16 blocks");
    __shared__ __attribute__((aligned(16))) float a[kCholNB][kCholNB + 4];
    __shared__ int s_bad;
    if (*info != 0) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // thread (i, h): row i = tid & 127 of columns h, h + 2, h + 4, ... (coalesced
    // over i), 16 loads in flight per batch
    // (every load unconditional, from inside the kb x kb block: the rows and
    // columns past kb read its last row / column and are replaced after)
    const int li = tid & (kCholNB - 1), lh = tid >> 7;
    const float *colp = A + min(li, kb - 1);
    for (int j0 = 0; j0 < kCholNB; j0 += 32) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = colp[(int64_t)min(j0 + 2 * u + lh, kb - 1) * ld];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int j = j0 + 2 * u + lh;
            a[li][j] = (li < kb && j < kb && li >= j) ? v[u] : (li == j ? 1.0f : 0.0f);
        }
    }
    if (tid == 0) s_bad = 0;
    __syncthreads();
    const int fi = lane & 15, fk = lane >> 4;   // operand lane map: A[fi][fk], B[fk][fi]; C row 4 fk + v, col fi
    for (int jb = 0; jb < kCholNB; jb += kCholPW) {
        if (jb > 0) {
            // the panel's columns jb .. jb + 15, rows jb .. 127, from every
            // factored column 0 .. jb - 1: one MFMA chain per 16 x 16 block
            for (int q = wave; q < (kCholNB - jb) / 16; q += 4) {
                const int i0 = jb + 16 * q;
                f32x4_t acc;
#pragma unroll
                for (int v = 0; v < 4; ++v) acc[v] = a[i0 + 4 * fk + v][jb + fi];
                for (int k16 = 0; k16 < jb; k16 += 16) {
                    float av[4], bv[4];
#pragma unroll
                    for (int kk = 0; kk < 4; ++kk) {
                        av[kk] = -a[i0 + fi][k16 + 4 * kk + fk];
                        bv[kk] = a[jb + fi][k16 + 4 * kk + fk];
                    }
#pragma unroll
                    for (int kk = 0; kk < 4; ++kk) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kk], bv[kk], acc, 0, 0, 0);
                }
#pragma unroll
                for (int v = 0; v < 4; ++v) a[i0 + 4 * fk + v][jb + fi] = acc[v];
            }
            __syncthreads();
        }
        {
            // the panel on all four waves: every wave factors the panel's top
            // 16 x 16 triangle in lanes 0-15 (the pivot rows its other lanes
            // need) and 48 of the rows below it in lanes 16-63; wave 0 writes
            // the triangle.  Each row sees the same operations as on one wave.
            const int r = lane < 16 ? jb + lane : jb + 16 + 48 * wave + (lane - 16);
            const int q = min(r, kCholNB - 1);
            float p0[kCholPW];
#pragma unroll
            for (int c4 = 0; c4 < kCholPW / 4; ++c4) {
                const float4 u0 = reinterpret_cast<const float4 *>(&a[q][jb])[c4];
                p0[4 * c4] = u0.x; p0[4 * c4 + 1] = u0.y; p0[4 * c4 + 2] = u0.z; p0[4 * c4 + 3] = u0.w;
            }
            __syncthreads();   // (every wave has read the triangle before wave 0 writes it)
            int bad = 0;
#pragma unroll
            for (int c = 0; c < kCholPW; ++c) {
                // (no early exit inside the unrolled panel: a failed pivot is
                // recorded and the rest of the panel computes garbage that the
                // block never stores)
                const int j = jb + c;
                const float djj = lane_value(p0[c], c);   // row j is lane c's
                // (pivots below FLT_MIN fail too: v_rsq_f32 of a denormal may overflow)
                if (bad == 0 && (!(djj >= 1.17549435e-38f) || !(djj < __builtin_huge_valf()))) bad = j + 1;
                const float rs = __builtin_amdgcn_rsqf(djj);
                p0[c] = p0[c] * rs;
#pragma unroll
                for (int c2 = c + 1; c2 < kCholPW; ++c2) {
                    const float lc2 = lane_value(p0[c], c2);   // L[jb + c2][j], lane c2's (already scaled)
                    p0[c2] = fmaf(-p0[c], lc2, p0[c2]);
                }
            }
            if (r < kCholNB && (lane >= 16 || wave == 0)) {
#pragma unroll
                for (int c = 0; c < kCholPW; ++c) a[r][jb + c] = p0[c];
            }
            if (tid == 0 && bad) s_bad = bad;
        }
        __syncthreads();
        if (s_bad) break;
    }
    if (s_bad) {
        if (tid == 0) atomicCAS(info, 0, (int)(k0 + s_bad));
        return;
    }
    float *colw = A + li + (int64_t)lh * ld;
    for (int j0 = 0; j0 < kCholNB; j0 += 32) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = a[li][j0 + 2 * u + lh];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int j = j0 + 2 * u + lh;
            if (li < kb && j < kb && li >= j) colw[(int64_t)(j0 + 2 * u) * ld] = v[u];
        }
    }
}

// The blocked Cholesky's trailing updates (a2): C[r][c] -= sum_k P[r][k] Q[c][k]
// over 128 x 128 tiles of C (all tiles of an m x nc block, or, lower != 0,
// the tiles on and below the diagonal of an m x m block), f32 in and out,
// column-major with leading dimension ld, K columns of P and Q.  The products
// on the matrix cores (v_mfma_f32_16x16x4_f32: exact f32 products, bit for
// bit a k-ordered fmaf chain) with C itself as the accumulator's start, so
// every element sees fmaf(-P[r][k], Q[c][k], C) in k order, as in a
// right-looking factorization.  rocBLAS ssyrk / sgemm ran these at 55-75 TF
// (tools/r3_gemm_probe.cpp).  Workgroup: 4 waves as 2 x 2 of 64 x 64; the
// MFMA's A side takes Q (the tile's columns) and its B side P (rows), so a
// lane's result column is a row of C: the stores run down C's columns.
// K in chunks of 32 staged through LDS as [k][row] (row stride 144 floats:
// the 16 rows x 4 k of one fragment read hit 64 distinct banks), double
// buffered, the next chunk's global loads in flight during the MFMAs.
constexpr int kUpBM = 128, kUpBK = 32, kUpLd = kUpBM + 16;
__global__ __launch_bounds__(256, 2) void chol_update_kernel(const float *__restrict__ P, const float *__restrict__ Q,
                                                             int64_t ld, int m, int nc, int K, int lower,
                                                             float *__restrict__ C) {
    __shared__ float Ps[2][kUpBK][kUpLd], Qs[2][kUpBK][kUpLd];
    int ti, tj;
    if (lower) {
        const int q = blockIdx.x;
        ti = (int)((sqrtf(8.0f * (float)q + 1.0f) - 1.0f) * 0.5f);
        while ((ti + 1) * (ti + 2) / 2 <= q) ++ti;
        while (ti * (ti + 1) / 2 > q) --ti;
        tj = q - ti * (ti + 1) / 2;
    } else {
        const int ntj = (nc + kUpBM - 1) / kUpBM;
        ti = blockIdx.x / ntj;
        tj = blockIdx.x % ntj;
    }
    const int r0 = ti * kUpBM, c0 = tj * kUpBM;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wr = wave >> 1, wc = wave & 1;
    // loader: row (tid & 127) of the chunk's k = (tid >> 7) + 2 u, u < 16, for P and Q
    const int lrow = tid & (kUpBM - 1), lk = tid >> 7;
    const bool prow = r0 + lrow < m, qrow = c0 + lrow < nc;
    const float *pp = P + (prow ? r0 + lrow : 0), *qp = Q + (qrow ? c0 + lrow : 0);
    float vp[16], vq[16];
    auto gload = [&](int k0) {
        // (K is a multiple of kUpBK: every k in range; rows past m / nc read
        // row 0 and are zeroed)
        const float *p0 = pp + (int64_t)(k0 + lk) * ld, *q0 = qp + (int64_t)(k0 + lk) * ld;
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const float a = p0[(int64_t)(2 * u) * ld], c = q0[(int64_t)(2 * u) * ld];
            vp[u] = prow ? a : 0.0f;
            vq[u] = qrow ? c : 0.0f;
        }
    };
    auto lstore = [&](int b) {
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            Ps[b][lk + 2 * u][lrow] = vp[u];
            Qs[b][lk + 2 * u][lrow] = vq[u];
        }
    };
    // accumulators from C: acc[cb][rb] holds C[r0 + 64 wr + 16 rb + (lane & 15)][c0 + 64 wc + 16 cb + 4 (lane >> 4) + v]
    const int fr = lane & 15, fg = lane >> 4;
    // a tile inside the block (uniform) needs no per-element tests
    const bool interior = r0 + kUpBM <= m && c0 + kUpBM <= nc;
    float *cw = C + (int64_t)(r0 + 64 * wr + fr) + (int64_t)(c0 + 64 * wc + 4 * fg) * ld;
    f32x4_t acc[4][4];
    if (interior) {
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
#pragma unroll
            for (int rb = 0; rb < 4; ++rb)
#pragma unroll
                for (int v = 0; v < 4; ++v) acc[cb][rb][v] = cw[16 * rb + (int64_t)(16 * cb + v) * ld];
    } else {
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
#pragma unroll
            for (int rb = 0; rb < 4; ++rb) {
                const int r = r0 + 64 * wr + 16 * rb + fr;
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const int c = c0 + 64 * wc + 16 * cb + 4 * fg + v;
                    acc[cb][rb][v] = (r < m && c < nc) ? cw[16 * rb + (int64_t)(16 * cb + v) * ld] : 0.0f;
                }
            }
    }
    gload(0);
    lstore(0);
    __syncthreads();
    const int nchunk = K / kUpBK;
    for (int ch = 0; ch < nchunk; ++ch) {
        const int b = ch & 1;
        if (ch + 1 < nchunk) gload((ch + 1) * kUpBK);
#pragma unroll
        for (int kk = 0; kk < kUpBK / 4; ++kk) {
            const int k = 4 * kk + fg;
            float qa[4], pb[4];
#pragma unroll
            for (int cb = 0; cb < 4; ++cb) qa[cb] = Qs[b][k][64 * wc + 16 * cb + fr];
#pragma unroll
            for (int rb = 0; rb < 4; ++rb) pb[rb] = -Ps[b][k][64 * wr + 16 * rb + fr];
#pragma unroll
            for (int cb = 0; cb < 4; ++cb)
#pragma unroll
                for (int rb = 0; rb < 4; ++rb)
                    acc[cb][rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(qa[cb], pb[rb], acc[cb][rb], 0, 0, 0);
        }
        if (ch + 1 < nchunk) lstore(b ^ 1);
        __syncthreads();
    }
    if (interior) {
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
#pragma unroll
            for (int rb = 0; rb < 4; ++rb)
#pragma unroll
                for (int v = 0; v < 4; ++v) cw[16 * rb + (int64_t)(16 * cb + v) * ld] = acc[cb][rb][v];
    } else {
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
#pragma unroll
            for (int rb = 0; rb < 4; ++rb) {
                const int r = r0 + 64 * wr + 16 * rb + fr;
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const int c = c0 + 64 * wc + 16 * cb + 4 * fg + v;
                    if (r < m && c < nc) cw[16 * rb + (int64_t)(16 * cb + v) * ld] = acc[cb][rb][v];
                }
            }
    }
}

// The blocked Cholesky's panel (a2): A21 := A21 L11^-T for the m2 x kb panel
// below a factored kb x kb diagonal block (rocBLAS strsm right / lower /
// transpose ran as ~10 launches, ~100 us per step, on the factorization's
// critical path).  Forward substitution row by row, x L11^T = a: 128 panel
// rows per workgroup, two threads per row (t and t + 128, one wave per SIMD);
// L11 row-major in LDS (stride 132: a row's 16-column blocks are aligned
// float4 reads, every lane reading the same address -- broadcast), the rows
// being solved in LDS column-major (lane-linear, conflict-free).
// Right-looking in 16-column blocks: both threads of a row solve the block's
// 16 values in registers, x_j = (a_j - sum_{u<j} x_u L_ju) * (1 / L_jj)
// (ascending u; the block of L read into registers first so that the chain
// waits on no LDS read), then each takes every other later column and
// subtracts the block's 16 terms.  Each x_j sees its terms in ascending
// column order, as in the plain forward substitution; the reciprocal of the
// pivot is the one extra rounding strsm's inverted diagonal has too.  kb <
// 128 (the last step) pads L11 with the identity.
constexpr int kTrsmLd = 132;
__global__ __launch_bounds__(256) void chol_trsm_kernel(const float *__restrict__ L11, int64_t ld, int kb,
                                                        float *__restrict__ A21, int64_t m2) {
    __shared__ __attribute__((aligned(16))) float Ls[kCholNB * kTrsmLd];
    __shared__ float X[kCholNB * kCholNB];
    SBO_CSTAMP(8);
    const int tid = threadIdx.x, t = tid & (kCholNB - 1), h = tid >> 7;
    const int64_t row = (int64_t)blockIdx.x * kCholNB + t;
    const bool in = row < m2;
    // columns of L11 and of the panel rows (coalesced over t), 16 columns of
    // loads in flight at a time, half the columns per thread of the pair;
    // identity padding past kb
    // (one predicate per thread for the loads, so all 16 of a batch are in
    // flight together; the upper triangle and the padding are fixed up after)
    const bool lin = t < kb;
    for (int j0 = 8 * h; j0 < kCholNB; j0 += 16) {
        float lv[8], xv[8];
        if (j0 + 8 <= kb) {
            if (lin) {
#pragma unroll
                for (int u = 0; u < 8; ++u) lv[u] = L11[t + (int64_t)(j0 + u) * ld];
            }
            if (in) {
#pragma unroll
                for (int u = 0; u < 8; ++u) xv[u] = A21[row + (int64_t)(j0 + u) * ld];
            }
        } else {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                lv[u] = (lin && j0 + u < kb) ? L11[t + (int64_t)(j0 + u) * ld] : 0.0f;
                xv[u] = (in && j0 + u < kb) ? A21[row + (int64_t)(j0 + u) * ld] : 0.0f;
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int j = j0 + u;
            Ls[t * kTrsmLd + j] = (j < kb && lin && t >= j) ? lv[u] : (t == j && j >= kb ? 1.0f : 0.0f);
            X[j * kCholNB + t] = (in && j < kb) ? xv[u] : 0.0f;
        }
    }
    __syncthreads();
    SBO_CSTAMP(9);
    for (int B = 0; B < kCholNB / 16; ++B) {
        const int j0 = 16 * B;
        // the 16 x 16 diagonal block of L (lower: row q needs q + 1 values)
        float4 lb[16][4];
#pragma unroll
        for (int q = 0; q < 16; ++q)
#pragma unroll
            for (int v = 0; v < 4; ++v)
                if (4 * v <= q) lb[q][v] = reinterpret_cast<const float4 *>(Ls + (j0 + q) * kTrsmLd + j0)[v];
        float xb[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) xb[u] = X[(j0 + u) * kCholNB + t];
        float rinv[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const float4 d = lb[q][q >> 2];
            rinv[q] = __fdiv_rn(1.0f, (q & 3) == 0 ? d.x : (q & 3) == 1 ? d.y : (q & 3) == 2 ? d.z : d.w);
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            float s = xb[q];
#pragma unroll
            for (int u = 0; u < q; ++u) {
                const float4 l4 = lb[q][u >> 2];
                const float l = (u & 3) == 0 ? l4.x : (u & 3) == 1 ? l4.y : (u & 3) == 2 ? l4.z : l4.w;
                s = fmaf(-xb[u], l, s);
            }
            xb[q] = s * rinv[q];
        }
        __syncthreads();   // every read of this block's columns is done
        if (h == 0) {
#pragma unroll
            for (int u = 0; u < 16; ++u) X[(j0 + u) * kCholNB + t] = xb[u];
        }
        // later columns of this thread (every other one), four at a time:
        // four independent FMA chains in flight instead of one
        for (int c0 = j0 + 16 + h; c0 < kCholNB; c0 += 8) {
            float v[4];
            float lv[4][16];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int c = min(c0 + 2 * k, kCholNB - 1);
                const float4 *lr = reinterpret_cast<const float4 *>(Ls + c * kTrsmLd + j0);
#pragma unroll
                for (int q4 = 0; q4 < 4; ++q4) {
                    const float4 l4 = lr[q4];
                    lv[k][4 * q4] = l4.x;
                    lv[k][4 * q4 + 1] = l4.y;
                    lv[k][4 * q4 + 2] = l4.z;
                    lv[k][4 * q4 + 3] = l4.w;
                }
                v[k] = X[c * kCholNB + t];
            }
#pragma unroll
            for (int u = 0; u < 16; ++u)
#pragma unroll
                for (int k = 0; k < 4; ++k) v[k] = fmaf(-xb[u], lv[k][u], v[k]);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (c0 + 2 * k < kCholNB) X[(c0 + 2 * k) * kCholNB + t] = v[k];
        }
        __syncthreads();
    }
    SBO_CSTAMP(10);
    if (in)
        for (int j = h; j < kb; j += 2) A21[row + (int64_t)j * ld] = X[j * kCholNB + t];
    SBO_CSTAMP(11);
}

// The same panel solve with the later columns' updates on the matrix cores
// (chol_trsm_kernel's default replacement).  Per 16-column block: the rows
// solve the block in registers, right-looking -- after x_q, every later s_q'
// of the block takes fmaf(-x_q, L[q'][q], s_q'), so each s still sees its
// terms in ascending column order, as in the forward substitution -- with the
// pivots' reciprocals computed once per workgroup; then the block's rank-16
// update of the later columns, X[c][t] -= sum_u L[c][u] x_u(t), as
// v_mfma_f32_16x16x4_f32 (a k-ordered fmaf chain from X itself: the same
// terms in the same order as chol_trsm_kernel's VALU loop, so the panel is
// bitwise the same).  The MFMA's A side takes L (result rows = columns c of
// X), its B side the solved x (result columns = panel rows t, contiguous in
// X's [c][t] layout, row stride 132: conflict-free result reads and writes).
// The block of L11 and the 128 panel rows in: two batches of 64 loads per
// thread in flight.
constexpr int kTrX = kCholNB + 4;
__global__ __launch_bounds__(256) void chol_trsm_mfma_kernel(const float *__restrict__ L11, int64_t ld, int kb,
                                                             float *__restrict__ A21, int64_t m2) {
    __shared__ __attribute__((aligned(16))) float Ls[kCholNB * kTrsmLd];
    __shared__ float X[kCholNB * kTrX];
    __shared__ float rinv[kCholNB];
    SBO_CSTAMP(8);
    const int tid = threadIdx.x, t = tid & (kCholNB - 1), h = tid >> 7;
    const int lane = tid & 63, wave = tid >> 6;
    const int64_t row = (int64_t)blockIdx.x * kCholNB + t;
    const bool in = row < m2, lin = t < kb;
    // loads: thread (t, h) takes columns h, h + 2, ... of L11's row t and of panel row t
    // (every load unconditional, clamped into the block; padding replaced below)
    const float *lp = L11 + min(t, kb - 1);
    const float *xp = A21 + (in ? row : 0);
    for (int jb = 0; jb < kCholNB; jb += 64) {
        float lv[32], xv[32];
#pragma unroll
        for (int u = 0; u < 32; ++u) {
            const int64_t off = (int64_t)min(jb + 2 * u + h, kb - 1) * ld;
            lv[u] = lp[off];
            xv[u] = xp[off];
        }
#pragma unroll
        for (int u = 0; u < 32; ++u) {
            const int j = jb + 2 * u + h;
            Ls[t * kTrsmLd + j] = (j < kb && lin && t >= j) ? lv[u] : (t == j && j >= kb ? 1.0f : 0.0f);
            X[j * kTrX + t] = (in && j < kb) ? xv[u] : 0.0f;
        }
    }
    __syncthreads();
    if (tid < kCholNB) rinv[tid] = __fdiv_rn(1.0f, Ls[tid * kTrsmLd + tid]);
    __syncthreads();
    SBO_CSTAMP(9);
    const int fr = lane & 15, fg = lane >> 4;
    for (int B = 0; B < kCholNB / 16; ++B) {
        const int j0 = 16 * B;
        if (h == 0) {
            // the block's 16 x 16 lower triangle of L (broadcast reads)
            float4 lb[16][4];
#pragma unroll
            for (int q = 0; q < 16; ++q)
#pragma unroll
                for (int v = 0; v < 4; ++v)
                    if (4 * v <= q) lb[q][v] = reinterpret_cast<const float4 *>(Ls + (j0 + q) * kTrsmLd + j0)[v];
            float sb[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) sb[q] = X[(j0 + q) * kTrX + t];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                sb[q] = sb[q] * rinv[j0 + q];
#pragma unroll
                for (int q2 = q + 1; q2 < 16; ++q2) {
                    const float4 l4 = lb[q2][q >> 2];
                    const float l = (q & 3) == 0 ? l4.x : (q & 3) == 1 ? l4.y : (q & 3) == 2 ? l4.z : l4.w;
                    sb[q2] = fmaf(-sb[q], l, sb[q2]);
                }
            }
#pragma unroll
            for (int q = 0; q < 16; ++q) X[(j0 + q) * kTrX + t] = sb[q];
        }
        __syncthreads();
        // rank-16 update of the later columns: 16 x 16 result blocks (column
        // block ci, row block ri), spread over the four waves
        const int c1 = j0 + 16, nci = (kCholNB - c1) / 16, nblk = nci * (kCholNB / 16);
        for (int qb = wave; qb < nblk; qb += 4) {
            const int ci = qb / (kCholNB / 16), ri = qb % (kCholNB / 16);
            const int cb0 = c1 + 16 * ci, rb0 = 16 * ri;
            f32x4_t acc;
#pragma unroll
            for (int v = 0; v < 4; ++v) acc[v] = X[(cb0 + 4 * fg + v) * kTrX + rb0 + fr];
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                const int u = 4 * kk + fg;
                const float av = -Ls[(cb0 + fr) * kTrsmLd + j0 + u];
                const float bv = X[(j0 + u) * kTrX + rb0 + fr];
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
            }
#pragma unroll
            for (int v = 0; v < 4; ++v) X[(cb0 + 4 * fg + v) * kTrX + rb0 + fr] = acc[v];
        }
        __syncthreads();
    }
    SBO_CSTAMP(10);
    if (in)
        for (int j = h; j < kb; j += 2) A21[row + (int64_t)j * ld] = X[j * kTrX + t];
    SBO_CSTAMP(11);
}

// The same panel solve, left-looking (round 5; SBO_OPT_CHOL_DIAG 1, the
// default -- 2 keeps the right-looking chol_trsm_mfma_kernel): before the
// rows solve 16-column block B, the four waves bring its columns up to date
// with every solved column 0 .. 16B - 1 in one MFMA chain per 16 x 16 result
// block, the accumulator in registers from X itself -- X[c][t] sees
// fmaf(-L[c][u], x_u(t), .) for u ascending, the same terms in the same order
// as the right-looking kernel's per-block updates (and the VALU kernel's
// loop), so the panel is bitwise the same; the right-looking kernel read and
// wrote every later block's accumulators through LDS after every block (56
// 16 x 16 updates per wave, each a four-MFMA chain) where this issues 8B
// MFMAs per wave as two interleaved chains.  Wave w owns row blocks 2w and
// 2w + 1 (rows 32w .. 32w + 31).
__global__ __launch_bounds__(256) void chol_trsm_ll_kernel(const float *__restrict__ L11, int64_t ld, int kb,
                                                           float *__restrict__ A21, int64_t m2) {
    __shared__ __attribute__((aligned(16))) float Ls[kCholNB * kTrsmLd];
    __shared__ float X[kCholNB * kTrX];
    __shared__ float rinv[kCholNB];
    const int tid = threadIdx.x, t = tid & (kCholNB - 1), h = tid >> 7;
    const int lane = tid & 63, wave = tid >> 6;
    const int64_t row = (int64_t)blockIdx.x * kCholNB + t;
    const bool in = row < m2, lin = t < kb;
    const float *lp = L11 + min(t, kb - 1);
    const float *xp = A21 + (in ? row : 0);
    for (int jb = 0; jb < kCholNB; jb += 64) {
        float lv[32], xv[32];
#pragma unroll
        for (int u = 0; u < 32; ++u) {
            const int64_t off = (int64_t)min(jb + 2 * u + h, kb - 1) * ld;
            lv[u] = lp[off];
            xv[u] = xp[off];
        }
#pragma unroll
        for (int u = 0; u < 32; ++u) {
            const int j = jb + 2 * u + h;
            Ls[t * kTrsmLd + j] = (j < kb && lin && t >= j) ? lv[u] : (t == j && j >= kb ? 1.0f : 0.0f);
            X[j * kTrX + t] = (in && j < kb) ? xv[u] : 0.0f;
        }
    }
    __syncthreads();
    if (tid < kCholNB) rinv[tid] = __fdiv_rn(1.0f, Ls[tid * kTrsmLd + tid]);
    __syncthreads();
    const int fr = lane & 15, fg = lane >> 4;
    const int rb0 = 32 * wave, rb1 = rb0 + 16;
    for (int B = 0; B < kCholNB / 16; ++B) {
        const int j0 = 16 * B;
        if (B > 0) {
            f32x4_t acc0, acc1;
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                acc0[v] = X[(j0 + 4 * fg + v) * kTrX + rb0 + fr];
                acc1[v] = X[(j0 + 4 * fg + v) * kTrX + rb1 + fr];
            }
            for (int k16 = 0; k16 < B; ++k16) {   // (16 columns at a time: operand reads batched)
                float av[4], b0[4], b1[4];
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    const int u = 16 * k16 + 4 * kk + fg;
                    av[kk] = -Ls[(j0 + fr) * kTrsmLd + u];
                    b0[kk] = X[u * kTrX + rb0 + fr];
                    b1[kk] = X[u * kTrX + rb1 + fr];
                }
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kk], b0[kk], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kk], b1[kk], acc1, 0, 0, 0);
                }
            }
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                X[(j0 + 4 * fg + v) * kTrX + rb0 + fr] = acc0[v];
                X[(j0 + 4 * fg + v) * kTrX + rb1 + fr] = acc1[v];
            }
            __syncthreads();
        }
        if (h == 0) {
            float4 lb[16][4];
#pragma unroll
            for (int q = 0; q < 16; ++q)
#pragma unroll
                for (int v = 0; v < 4; ++v)
                    if (4 * v <= q) lb[q][v] = reinterpret_cast<const float4 *>(Ls + (j0 + q) * kTrsmLd + j0)[v];
            float sb[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) sb[q] = X[(j0 + q) * kTrX + t];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                sb[q] = sb[q] * rinv[j0 + q];
#pragma unroll
                for (int q2 = q + 1; q2 < 16; ++q2) {
                    const float4 l4 = lb[q2][q >> 2];
                    const float l = (q & 3) == 0 ? l4.x : (q & 3) == 1 ? l4.y : (q & 3) == 2 ? l4.z : l4.w;
                    sb[q2] = fmaf(-sb[q], l, sb[q2]);
                }
            }
#pragma unroll
            for (int q = 0; q < 16; ++q) X[(j0 + q) * kTrX + t] = sb[q];
        }
        __syncthreads();
    }
    if (in)
        for (int j = h; j < kb; j += 2) A21[row + (int64_t)j * ld] = X[j * kTrX + t];
}

// Row 1-norms of the packed operand: block I, thread r sums |A[I*BM + r][:]|.
// Row 1-norms of the packed operand, |A[I*BM + r][:]|_1: block (c, I)
// sums row r over k-tiles [c*kRowL1Tiles, (c+1)*kRowL1Tiles) of row block I
// and adds into row_l1 (zeroed by the launcher).
constexpr int kRowL1Tiles = 4;
__global__ __launch_bounds__(kBM) void row_l1_kernel(const float *__restrict__ aug, int64_t I0,
                                                     double *__restrict__ row_l1) {
    const int64_t I = I0 + blockIdx.y;
    const int64_t kb0 = (int64_t)blockIdx.x * kRowL1Tiles;
    const int64_t nkb = (I + 1) * kTilesPerRowBlockStep;
    if (kb0 >= nkb) return;
    const int r = threadIdx.x;
    const float *t = aug + (tile_start(I) + kb0) * kTileFloats;
    double s = 0.0;
    for (int64_t kb = 0; kb < kRowL1Tiles && kb0 + kb < nkb; ++kb)
        for (int k = 0; k < kBK; ++k) s += fabs((double)t[kb * kTileFloats + tile_offset(k, r)]);
    atomicAdd(row_l1 + I * kBM + r, s);
}

// The split of an f32 value into three bf16 pieces, v = v0 + v1 + v2 (+ a
// remainder below 2^-24 |v|), exactly as pack_x3_kernel splits the operand
// (the same round-to-nearest-even conversion instruction).
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float bf16_rn(float a) {
    const f32x2_t v = {a, 0.0f};
    const uint32_t w = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
    return __uint_as_float(w << 16);
}

// Per packed tile, gain bounds (log2, rounded up), two float4 per tile:
// lgn[2T]   .x = log2(16 max_r |A_r|_1)  (|A k|_2 <= sqrt(256) |A k|_inf <= 16 max_r |A_r|_1 max|k|)
//           .y = log2 of a bound on the spectral norm ||A_It||_2  (|A k|_2 <= ||A||_2 |k|_2):
//                with the 64x64 Gram matrix G = A^T A (PSD, f64), ||A||_2^2 = lambda_max(G)
//                <= ||G^16||_inf^(1/16) (any induced norm bounds the spectral radius;
//                at most 64^(1/32) = 1.14x over ||A||_2 for a 64 x 64 G),
//                also <= |A|_F^2 = trace G; the smaller of the two;
//           .z = log2(|A_It|_F), which also bounds || |A_It| ||_2;
// lgn[2T+1] the same two bounds for the bf16 pieces the split sweep
//           multiplies (A = A0 + A1 + A2, pack_x3_kernel): .x, .y of A1 and
//           .z, .w of A2 (16 max row 1-norm, spectral) -- the products a
//           tile's lower precision levels leave out are A2 K0 + A1 K1 + A0 K2
//           (three products) and also A1 K0 + A0 K1 (one product), bounded
//           plane by plane in tile_increments.
// The plan pairs the row-sum bounds with the largest K* of the tile and the
// spectral ones with a bound on |k|_2 from the tile's points.  One workgroup
// per tile; the three matrices one after the other.  The Gram matrices and
// their squarings are bf16 MFMA products of split operands (below); wave w
// owns two or three of the ten lower 16 x 16 blocks of each 64 x 64 product.
// LDS row stride (floats) of the powers of G: 68 puts the row-sum pass's
// 16-B reads and the mirrored stores on distinct banks
constexpr int kTnGmLd = kBK + 4;
// Round 6: the Gram matrices from the tile's bf16 pieces on the bf16 matrix
// cores.  A = A0 + A1 + A2 (+ r, |r| < 2^-24 |A|) exactly as pack_x3_kernel
// splits it, so G1 = A1^T A1 and G2 = A2^T A2 are products of bf16 values --
// exact products, f32 accumulation -- and G = A^T A is taken as A0^T A0 + A0^T
// A1 + A1^T A0 + A0^T A2 + A2^T A0 + G1 (the dropped A1^T A2 + A2^T A1 + A2^T
// A2 and r's terms are < 2^-22 |A|^T|A|).  One v_mfma_f32_16x16x32_bf16 covers
// 16 x 16 x 32 where the f64 16x16x4 form needed eight at four times the
// cycles each.  Rigour: the stored G_c is symmetrised (lower blocks mirrored)
// and |G_c - G| <= delta |A|^T |A| entrywise with delta = 2^-16 (<= 80 f32
// roundings of partial sums of |A|^T |A|, 4.8e-6, plus the dropped terms),
// so ||G_c - G||_2 <= delta |A|_F^2 and, by Weyl, lambda_max(G) <=
// lambda_max(G_c) + delta |A|_F^2: the spectral bound below adds that term
// (at most 64 delta = 1e-3 relative, since ||A||_2^2 >= |A|_F^2 / 64).  The
// squarings run on the bf16 matrix cores too (their bound: in the kernel).  Row sums and |A|_F^2 come from the pieces in f64 (A0 +
// A1 + A2 = A to 2^-24: inside the outputs' 1e-5 log2 margin).  The pieces are
// those pack_x3_kernel cuts (the same instructions on the unscaled values),
// each scaled by its own power of two 2^s_p (exact) so that the piece's
// largest |entry| is in [1, 2): f32 products and sums then stay far above
// f32's underflow (unscaled, A2^T A2 of a tile of 2^-60 entries underflowed
// and the bound lost its rigour -- caught by comparing against the f64
// kernel's bounds).  The cross terms of G go to accumulators of their own
// and are combined in f64 with the exact scale factors.  What underflow
// remains is bounded by an absolute term: 2^-110 of each accumulator's own
// scale in ||G_c - G||_2 (64 x 264 operations below 2^-126 each).
// The tile is staged a quarter (64 rows) at a time: the quarter's floats are
// one contiguous 64 x 64 block in k-major order (tile_offset), and the Gram's
// contraction runs over that storage order (any order of the rows serves).
constexpr int kTnPq = kBK + 8;                 // bf16 per staged k row: 144 B, conflict-free b128 reads
constexpr double kTnDelta = 1.0 / 65536.0;     // 2^-16
typedef float f32x4_t2 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f32x4_t2 mfma_bf16(uint4 a, uint4 b, f32x4_t2 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                   c, 0, 0, 0);
}
// a 16 x 16 block (bi >= bj) of plane pi's symmetric 64 x 64 Gram matrix,
// scaled 2^(2 sp[pi]), from the f32 MFMA accumulators (lane l, element v:
// row 16 bi + 4 (l>>4) + v, column 16 bj + (l&15)): G_A = a00 + 2^(s0 - s1)
// a01 + 2^(s0 - s2) a02 + 2^(2 (s0 - s1)) a1 in f64 (exact scalings); the
// entries above the diagonal of a diagonal block are left 0 (the stores
// mirror the lower ones)
__device__ __forceinline__ void gram_values(double (&x)[4], int bi, int bj, int lane, int pi, f32x4_t2 a00,
                                            f32x4_t2 a01, f32x4_t2 a02, f32x4_t2 a1, f32x4_t2 a2,
                                            const int (&sp)[3]) {
    const double c01 = ldexp(1.0, sp[0] - sp[1]), c02 = ldexp(1.0, sp[0] - sp[2]), c11 = c01 * c01;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        const int i = 16 * bi + 4 * (lane >> 4) + v, j = 16 * bj + (lane & 15);
        x[v] = (bi != bj || i >= j)
                   ? (pi == 0 ? (((double)a00[v] + c01 * (double)a01[v]) + c02 * (double)a02[v]) + c11 * (double)a1[v]
                              : (pi == 1 ? (double)a1[v] : (double)a2[v]))
                   : 0.0;
    }
}
// an f32 block (bi >= bj) of a symmetric matrix into gf (stride kTnGmLd):
// the lower entries and their mirror (a diagonal block's upper entries from
// its lower ones, so the stored matrix is exactly symmetric); the mirror of
// a lane's four rows is one 16-B store
__device__ __forceinline__ void store_sym_f32(float *gf, int bi, int bj, int lane, const float (&x)[4]) {
    const int i0 = 16 * bi + 4 * (lane >> 4), j = 16 * bj + (lane & 15);
    if (bi != bj) {
#pragma unroll
        for (int v = 0; v < 4; ++v) gf[(i0 + v) * kTnGmLd + j] = x[v];
        *reinterpret_cast<float4 *>(gf + j * kTnGmLd + i0) = make_float4(x[0], x[1], x[2], x[3]);
    } else {
#pragma unroll
        for (int v = 0; v < 4; ++v)
            if (i0 + v >= j) {
                gf[(i0 + v) * kTnGmLd + j] = x[v];
                gf[j * kTnGmLd + i0 + v] = x[v];
            }
    }
}
// FUSED (round 6): the tile is first packed here from the f64 inverse --
// pack_operand_kernel's values, (float)(sf2 L^-1), written to aug -- so the
// pack and the norms are one pass over L^-1 (the staging pass re-reads the
// thread's own stores from L2).
template <bool FUSED>
__global__ __launch_bounds__(kBM, 2) void tile_norm_kernel(const float *__restrict__ aug, int64_t t0,
                                                           float4 *__restrict__ lgn, const double *__restrict__ Linv,
                                                           int64_t ld, int64_t n, double sf2, float *augw) {
    __shared__ __attribute__((aligned(16))) unsigned short pq[3][kBK * kTnPq];   // a quarter's pieces [k][c] (27 KiB)
    __shared__ __attribute__((aligned(16))) float gm[kBK * kTnGmLd];   // G, then its powers, normalised f32 (17 KiB)
    __shared__ double rpart[3][4][kBK];        // row-sum partials of a quarter (6 KiB)
    __shared__ double red[2][kBM / 64];
    __shared__ double fred[3][kBM / 64], rwm[3][kBM / 64];   // per wave: |.|_F^2 sums, row-sum maxima
    const int64_t tile = t0 + blockIdx.x;
    const float *t = aug + tile * kTileFloats;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    __shared__ float out[6];                     // (rows, spectral) of A; of A1; of A2 (LDS: a plane-indexed array)
    double lg_fro_a = -1000.0;
    // this wave's lower blocks of the 4 x 4 block grid of G: (0,0) (1,0) (1,1) |
    // (2,0) (2,1) (2,2) | (3,0) (3,1) | (3,2) (3,3)
    const int nb = wave < 2 ? 3 : 2;
    const int tbi[3] = {wave < 2 ? 2 * wave : 3, wave < 2 ? 2 * wave + (wave == 0 ? 1 : 0) : 3, wave == 0 ? 1 : 2};
    const int tbj[3] = {wave < 3 ? 0 : 2, wave == 0 ? 0 : (wave == 1 ? 1 : (wave == 2 ? 1 : 3)), wave == 0 ? 1 : 2};
    // the Gram accumulators: A (its five cross terms), A1, A2
    // G_A's terms A0^T A0, A1^T A0 + A0^T A1, A2^T A0 + A0^T A2 (scaled 2^(s0 + s_p)), then G1, G2
    f32x4_t2 acc00[3], acc01[3], acc02[3], acc1[3], acc2[3];
#pragma unroll
    for (int b = 0; b < 3; ++b) acc00[b] = acc01[b] = acc02[b] = acc1[b] = acc2[b] = f32x4_t2{0.f, 0.f, 0.f, 0.f};
    double rmax[3] = {0.0, 0.0, 0.0}, fro[3] = {0.0, 0.0, 0.0};
    const int sk = tid >> 2, sc = 16 * (tid & 3);   // staging: k row sk, storage columns sc .. sc + 15
    const int rc = tid & 63, rk = tid >> 6;         // row sums: column rc, k in [16 rk, 16 rk + 16)
    // the thread's 16 floats of each quarter (a quarter is one contiguous
    // 64 x 64 block), all in flight at once; the tile's largest |entry| sets
    // the scale 2^sc
    // (the tile is read twice, the second time from L2: a pass for the
    // pieces' maxima, then the staging)
    auto load16 = [&](int q, float (&v)[16]) {
        const float4 *src = FUSED ? reinterpret_cast<const float4 *>(augw + tile * kTileFloats + q * 64 * kBK + 16 * tid)
                                  : reinterpret_cast<const float4 *>(t + q * 64 * kBK + 16 * tid);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float4 f = src[j];
            v[4 * j] = f.x;
            v[4 * j + 1] = f.y;
            v[4 * j + 2] = f.z;
            v[4 * j + 3] = f.w;
        }
    };
    __shared__ float pmax[3][kBM / 64];
    {
        float amax[3] = {0.0f, 0.0f, 0.0f};
        // FUSED: the tile's row block and k-tile (tile = tile_start(I) + kb)
        int64_t fI = 0, fkb = 0;
        if (FUSED) {
            fI = (int64_t)((sqrt(1.0 + 2.0 * (double)tile) - 1.0) * 0.5);
            while (fI > 0 && tile_start(fI) > tile) --fI;
            while (tile_start(fI + 1) <= tile) ++fI;
            fkb = tile - tile_start(fI);
        }
#pragma unroll
        for (int q = 0; q < kBM / 64; ++q) {
            float tv[16];
            if (FUSED) {
                // element 16 tid + j of quarter q (tile_offset): k = tid / 4, row
                // 64 q + 16 (j & 3) + 4 (tid & 3) + j / 4 -- pack_operand_kernel's value
                const int64_t col = fkb * kBK + (tid >> 2);
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const int64_t row = fI * kBM + 64 * q + 16 * (j & 3) + 4 * (tid & 3) + (j >> 2);
                    tv[j] = (row < n && col < n && col <= row) ? (float)(sf2 * Linv[row + col * ld]) : 0.0f;
                }
                float4 *dst = reinterpret_cast<float4 *>(augw + tile * kTileFloats + q * 64 * kBK + 16 * tid);
#pragma unroll
                for (int j = 0; j < 4; ++j) dst[j] = make_float4(tv[4 * j], tv[4 * j + 1], tv[4 * j + 2], tv[4 * j + 3]);
            } else {
                load16(q, tv);
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const float x = tv[j];
                const float a0 = bf16_rn(x), r1 = x - a0, a1 = bf16_rn(r1), a2 = bf16_rn(r1 - a1);
                amax[0] = fmaxf(amax[0], fabsf(a0));
                amax[1] = fmaxf(amax[1], fabsf(a1));
                amax[2] = fmaxf(amax[2], fabsf(a2));
            }
        }
#pragma unroll
        for (int pc = 0; pc < 3; ++pc) {
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) amax[pc] = fmaxf(amax[pc], __shfl_xor(amax[pc], o));
            if (lane == 0) pmax[pc][wave] = amax[pc];
        }
    }
    __syncthreads();
    int sp[3];           // the pieces' scales: 2^sp max |piece| in [1, 2)
    float up[3];
    double dn[3];
#pragma unroll
    for (int pc = 0; pc < 3; ++pc) {
        const float m = fmaxf(fmaxf(pmax[pc][0], pmax[pc][1]), fmaxf(pmax[pc][2], pmax[pc][3]));
        sp[pc] = m > 0.0f ? -ilogbf(m) : 0;
        up[pc] = ldexpf(1.0f, sp[pc]);
        dn[pc] = ldexp(1.0, -sp[pc]);
    }
#pragma unroll 1
    for (int q = 0; q < kBM / 64; ++q) {
        // stage: split (as pack_x3_kernel does, unscaled), scale each piece by 2^sp (exact), store
        {
            float tv[16];
            load16(q, tv);
            uint32_t w[3][8];
#pragma unroll
            for (int j = 0; j < 16; j += 2) {
                uint32_t h[3][2];
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const float x = tv[j + e];
                    const float a0 = bf16_rn(x), r1 = x - a0, a1 = bf16_rn(r1), a2 = bf16_rn(r1 - a1);
                    h[0][e] = __float_as_uint(a0 * up[0]) >> 16;
                    h[1][e] = __float_as_uint(a1 * up[1]) >> 16;
                    h[2][e] = __float_as_uint(a2 * up[2]) >> 16;
                }
#pragma unroll
                for (int pc = 0; pc < 3; ++pc) w[pc][j / 2] = h[pc][0] | (h[pc][1] << 16);
            }
#pragma unroll
            for (int pc = 0; pc < 3; ++pc) {
                uint4 *dst = reinterpret_cast<uint4 *>(pq[pc] + sk * kTnPq + sc);
                dst[0] = make_uint4(w[pc][0], w[pc][1], w[pc][2], w[pc][3]);
                dst[1] = make_uint4(w[pc][4], w[pc][5], w[pc][6], w[pc][7]);
            }
        }
        __syncthreads();
        // Gram: two 32-deep contraction steps over the quarter's 64 storage columns
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int co = 32 * ks + 8 * (lane >> 4);
            uint4 fa[3][3], fb[3][3];   // [piece][block]
#pragma unroll
            for (int b = 0; b < 3; ++b)
                if (b < nb)
#pragma unroll
                    for (int pc = 0; pc < 3; ++pc) {
                        fa[pc][b] = *reinterpret_cast<const uint4 *>(pq[pc] + (16 * tbi[b] + (lane & 15)) * kTnPq + co);
                        fb[pc][b] = *reinterpret_cast<const uint4 *>(pq[pc] + (16 * tbj[b] + (lane & 15)) * kTnPq + co);
                    }
#pragma unroll
            for (int b = 0; b < 3; ++b)
                if (b < nb) {
                    acc02[b] = mfma_bf16(fa[0][b], fb[2][b], mfma_bf16(fa[2][b], fb[0][b], acc02[b]));
                    acc01[b] = mfma_bf16(fa[0][b], fb[1][b], mfma_bf16(fa[1][b], fb[0][b], acc01[b]));
                    acc00[b] = mfma_bf16(fa[0][b], fb[0][b], acc00[b]);
                    acc1[b] = mfma_bf16(fa[1][b], fb[1][b], acc1[b]);
                    acc2[b] = mfma_bf16(fa[2][b], fb[2][b], acc2[b]);
                }
        }
        // row sums (the quarter's 64 rows = its 64 storage columns) and |.|_F^2,
        // in f64 from the pieces (A = A0 + A1 + A2 to 2^-24)
        {
            double s[3] = {0.0, 0.0, 0.0};
#pragma unroll 4
            for (int k = 16 * rk; k < 16 * rk + 16; ++k) {
                // (unscaled: exact powers of two)
                const double b0 = (double)__uint_as_float((uint32_t)pq[0][k * kTnPq + rc] << 16) * dn[0];
                const double b1 = (double)__uint_as_float((uint32_t)pq[1][k * kTnPq + rc] << 16) * dn[1];
                const double b2 = (double)__uint_as_float((uint32_t)pq[2][k * kTnPq + rc] << 16) * dn[2];
                const double a = b0 + b1 + b2;     // exact (three bf16 values of one f32's split)
                s[0] += fabs(a);
                s[1] += fabs(b1);
                s[2] += fabs(b2);
                fro[0] = fma(a, a, fro[0]);
                fro[1] = fma(b1, b1, fro[1]);
                fro[2] = fma(b2, b2, fro[2]);
            }
#pragma unroll
            for (int pc = 0; pc < 3; ++pc) rpart[pc][rk][rc] = s[pc];
        }
        __syncthreads();   // (pq restaged next quarter; rpart complete)
        if (rk == 0)
#pragma unroll
            for (int pc = 0; pc < 3; ++pc)
                rmax[pc] = fmax(rmax[pc], ((rpart[pc][0][rc] + rpart[pc][1][rc]) + rpart[pc][2][rc]) + rpart[pc][3][rc]);
    }
    // the block maxima of the row sums and the sums of |.|_F^2 (fixed-order
    // trees), unscaled (exact: powers of two)
#pragma unroll
    for (int pc = 0; pc < 3; ++pc) {
        double rs = rmax[pc], fs = fro[pc];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            rs = fmax(rs, __shfl_xor(rs, o));
            fs += __shfl_xor(fs, o);
        }
        if (lane == 0) {
            red[0][wave] = 0.0;
            fred[pc][wave] = fs;
            rwm[pc][wave] = rs;
        }
    }
    __syncthreads();
    double rowmax_all[3];
#pragma unroll
    for (int pc = 0; pc < 3; ++pc)
        rowmax_all[pc] = fmax(fmax(rwm[pc][0], rwm[pc][1]), fmax(rwm[pc][2], rwm[pc][3]));
#pragma unroll 1
    for (int pi = 0; pi < 3; ++pi) {
        const int plane = pi == 0 ? -1 : pi;     // -1: A itself, then A1, A2
        // the plane's Gram matrix G_c (f64, registers), normalised by its
        // largest entry's power of two 2^e0 and rounded to f32: M0, symmetric
        double gv[3][4];
        double gmx = 0.0;
#pragma unroll
        for (int b = 0; b < 3; ++b)
            if (b < nb) {
                gram_values(gv[b], tbi[b], tbj[b], lane, pi, acc00[b], acc01[b], acc02[b], acc1[b], acc2[b], sp);
#pragma unroll
                for (int v = 0; v < 4; ++v) gmx = fmax(gmx, fabs(gv[b][v]));
            }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) gmx = fmax(gmx, __shfl_xor(gmx, o));
        if (lane == 0) red[1][wave] = gmx;
        __syncthreads();
        const double mx0 = fmax(fmax(red[1][0], red[1][1]), fmax(red[1][2], red[1][3]));
        const int e0 = mx0 > 0.0 ? ilogb(mx0) : 0;
#pragma unroll
        for (int b = 0; b < 3; ++b)
            if (b < nb) {
                float xf[4];
#pragma unroll
                for (int v = 0; v < 4; ++v) xf[v] = (float)ldexp(gv[b][v], -e0);
                store_sym_f32(gm, tbi[b], tbj[b], lane, xf);
            }
        const double fro2 = ((fred[pi][0] + fred[pi][1]) + fred[pi][2]) + fred[pi][3];
        double s = rowmax_all[pi];
        // Four squarings on the bf16 matrix cores (round 6; f64 MFMA before,
        // 2.1 ms of the C4 fit's critical path): M_k is split into three bf16
        // planes as pack_x3_kernel splits (pq, free after the Gram), S_k =
        // M_k M_k is taken as the six products a2 b0 + a1 b1 + a0 b2 + a1 b0 + a0
        // b1 + a0 b0 (exact products, f32 accumulation) on the ten lower
        // blocks, and M_(k+1) = 2^-e S_k (e: S_k's largest entry's exponent,
        // exact) is stored mirrored, so every M_k is exactly symmetric.
        // Rigour: |S_k - M_k^2| <= eps |M_k| |M_k| entrywise with eps = 2^-15
        // (the dropped a1 b2 + a2 b1 + a2 b2 and the split's remainder < 2^-22,
        // <= 396 f32 roundings of partial sums of the |terms| < 2.4e-5), so
        // ||S_k - M_k^2||_2 <= eta ||M_k||_2^2 with eta = 64 eps (||
        // |M| |M| ||_2 <= |M|_F^2 <= 64 ||M||_2^2) and ||M_k||_2^2 <=
        // ||S_k||_2 / (1 - eta); M0 is G_c 2^-e0 rounded to f32, ||G_c||_2 <=
        // 2^e0 ||M0||_2 / (1 - 2^-21).  Chained: log2 ||G_c||_2 <= e0 + (T +
        // log2 ||M4||_inf + 15 log2(1 / (1 - eta))) / 16 + log2(1 / (1 - 2^-21)),
        // T = 8 e1 + 4 e2 + 2 e3 + e4 (||M4||_2 <= ||M4||_inf: symmetric).
        // Underflow (entries below 2^-110 of the largest) costs < 2^-90 of
        // ||S_k||_2 >= 1, inside eps's slack.
        constexpr int kGramSquarings = 4;
        constexpr double kSqEta = 64.0 / 32768.0;   // 64 eps, eps = 2^-15
        int T = 0;
        bool live = mx0 > 0.0;
        for (int it = 0; it < kGramSquarings && live; ++it) {
            __syncthreads();   // M_k stored (and every read of pq by the last products done)
            {
                // split M_k into the planes: row sk, columns sc .. sc + 15
                const float4 *src = reinterpret_cast<const float4 *>(gm + sk * kTnGmLd + sc);
                uint32_t w[3][8];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 f = src[q];
                    const float xv[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
                    for (int e = 0; e < 4; e += 2) {
                        uint32_t h[3][2];
#pragma unroll
                        for (int u = 0; u < 2; ++u) {
                            const float x = xv[e + u];
                            const float a0 = bf16_rn(x), r1 = x - a0, a1 = bf16_rn(r1), a2 = bf16_rn(r1 - a1);
                            h[0][u] = __float_as_uint(a0) >> 16;
                            h[1][u] = __float_as_uint(a1) >> 16;
                            h[2][u] = __float_as_uint(a2) >> 16;
                        }
#pragma unroll
                        for (int pc = 0; pc < 3; ++pc) w[pc][(4 * q + e) / 2] = h[pc][0] | (h[pc][1] << 16);
                    }
                }
#pragma unroll
                for (int pc = 0; pc < 3; ++pc) {
                    uint4 *dst = reinterpret_cast<uint4 *>(pq[pc] + sk * kTnPq + sc);
                    dst[0] = make_uint4(w[pc][0], w[pc][1], w[pc][2], w[pc][3]);
                    dst[1] = make_uint4(w[pc][4], w[pc][5], w[pc][6], w[pc][7]);
                }
            }
            __syncthreads();
            f32x4_t2 sq[3];
#pragma unroll
            for (int b = 0; b < 3; ++b) sq[b] = f32x4_t2{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const int co = 32 * ks + 8 * (lane >> 4);
                uint4 fa[3][3], fb[3][3];   // [piece][block]
#pragma unroll
                for (int b = 0; b < 3; ++b)
                    if (b < nb)
#pragma unroll
                        for (int pc = 0; pc < 3; ++pc) {
                            fa[pc][b] = *reinterpret_cast<const uint4 *>(pq[pc] + (16 * tbi[b] + (lane & 15)) * kTnPq + co);
                            fb[pc][b] = *reinterpret_cast<const uint4 *>(pq[pc] + (16 * tbj[b] + (lane & 15)) * kTnPq + co);
                        }
#pragma unroll
                for (int b = 0; b < 3; ++b)
                    if (b < nb) {
                        sq[b] = mfma_bf16(fa[2][b], fb[0][b], sq[b]);
                        sq[b] = mfma_bf16(fa[1][b], fb[1][b], sq[b]);
                        sq[b] = mfma_bf16(fa[0][b], fb[2][b], sq[b]);
                        sq[b] = mfma_bf16(fa[1][b], fb[0][b], sq[b]);
                        sq[b] = mfma_bf16(fa[0][b], fb[1][b], sq[b]);
                        sq[b] = mfma_bf16(fa[0][b], fb[0][b], sq[b]);
                    }
            }
            float qmx = 0.0f;
#pragma unroll
            for (int b = 0; b < 3; ++b)
                if (b < nb)
#pragma unroll
                    for (int v = 0; v < 4; ++v) qmx = fmaxf(qmx, fabsf(sq[b][v]));
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) qmx = fmaxf(qmx, __shfl_xor(qmx, o));
            if (lane == 0) red[0][wave] = (double)qmx;
            __syncthreads();   // every wave's maximum (and every read of gm by the split is done)
            const double mk = fmax(fmax(red[0][0], red[0][1]), fmax(red[0][2], red[0][3]));
            live = mk > 0.0;
            const int ek = live ? ilogb(mk) : 0;
            T = 2 * T + ek;
#pragma unroll
            for (int b = 0; b < 3; ++b)
                if (b < nb) {
                    // (the diagonal block's upper entries are computed too; only the lower are kept)
                    const float xf[4] = {ldexpf(sq[b][0], -ek), ldexpf(sq[b][1], -ek), ldexpf(sq[b][2], -ek),
                                         ldexpf(sq[b][3], -ek)};
                    store_sym_f32(gm, tbi[b], tbj[b], lane, xf);
                }
        }
        __syncthreads();   // the last power stored
        // ||M4||_inf: largest absolute row sum (f64)
        double rs = 0.0;
        if (tid < kBK)
            for (int j = 0; j < kBK; ++j) rs += fabs((double)gm[tid * kTnGmLd + j]);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) rs = fmax(rs, __shfl_xor(rs, o));
        if (lane == 0) red[1][wave] = rs;
        __syncthreads();
        rs = fmax(fmax(red[1][0], red[1][1]), fmax(red[1][2], red[1][3]));
        if (!live) rs = 0.0;   // (a zero Gram matrix)
        // log2 ||A||_2 (the plane scaled by 2^sp: G_c = 2^(2 sp) G) from the
        // chain above, 1e-6 for the f64 row sums and logs; then ||A||_2^2 <=
        // that^2 + delta |A|_F^2 (G_c's own error) + the absolute underflow
        // term: 2^-110 per accumulator at its own scale, five for G_A, all at
        // most 2^(-2 sp) unscaled
        const int spl = sp[pi];
        const double lg_g = (double)e0 +
                            ((double)T + log2(rs) - (double)((1 << kGramSquarings) - 1) * log2(1.0 - kSqEta)) /
                                (double)(1 << kGramSquarings) -
                            log2(1.0 - 0x1p-21);
        const double lg_pow = rs > 0.0 ? 0.5 * lg_g + 1e-6 - spl : -1000.0;
        const double spec2 = (rs > 0.0 ? exp2(2.0 * lg_pow) : 0.0) + kTnDelta * fro2 + ldexp(5.0, -110 - 2 * spl);
        const double lg_spec = spec2 > 0.0 ? 0.5 * log2(spec2) : -1000.0;
        const double lg_fro = fro2 > 0.0 ? 0.5 * log2(fro2) : -1000.0;
        const int o = 2 * pi;                    // A: 0, A1: 2, A2: 4
        if (tid == 0) {
            out[o] = s > 0.0 ? (float)log2(16.0 * s) + 1e-5f : -1000.0f;
            out[o + 1] = (float)fmin(lg_spec, lg_fro) + 1e-5f;
        }
        if (plane < 0) lg_fro_a = lg_fro;
        __syncthreads();   // gm / red / rsum / at are rewritten for the next matrix
    }
    if (tid == 0) {
        lgn[2 * tile] = make_float4(out[0], out[1], (float)lg_fro_a + 1e-5f, 0.0f);
        lgn[2 * tile + 1] = make_float4(out[2], out[3], out[4], out[5]);
    }
}

// d[i] = (double)in[i] - v
__global__ void widen_sub_kernel(const float *__restrict__ in, double v, int64_t n, double *__restrict__ d) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) d[i] = (double)in[i] - v;
}

__global__ void narrow_kernel(const double *__restrict__ d, int64_t n, float *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (float)d[i];
}

// Bounding box of each k-tile's valid training points: (xmin, xmax, ymin, ymax);
// a tile with no valid point gets an empty box (+inf, -inf, +inf, -inf).
__global__ void tile_box_kernel(const float *__restrict__ x, const float *__restrict__ y, int64_t n,
                                int64_t ntiles, float4 *__restrict__ kbox) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntiles) return;
    float x0 = INFINITY, x1 = -INFINITY, y0 = INFINITY, y1 = -INFINITY;
    for (int64_t k = t * kBK; k < (t + 1) * kBK && k < n; ++k) {
        x0 = fminf(x0, x[k]); x1 = fmaxf(x1, x[k]);
        y0 = fminf(y0, y[k]); y1 = fmaxf(y1, y[k]);
    }
    kbox[t] = make_float4(x0, x1, y0, y1);
}

// ---------------------------------------------------------- a3+a4 predict
// Work item (I, qb): the BN = 128 queries [qb*BN, qb*BN+BN) against row
// block I = rows [I*BM, I*BM+BM) of A = sf2 L^-1 (BM = 256), over the k-tiles
// t < 4(I+1) the tick's plan keeps.  A workgroup has eight waves, two per
// SIMD; wave w owns the 16 queries qb*BN + 16w + (l&15) and ALL 256 rows as
// sixteen 16-row blocks: sixteen accumulators of v_mfma_f32_16x16x4_f32
// (exact f32, 64 FLOP/clk/SIMD).  The B operand K*[k][q] is generated per
// lane -- lane l holds k = l>>4, q = l&15, exactly the MFMA B-fragment map --
// so K* never touches LDS or HBM.
//
// Why this shape: on gfx950 the VALU work of a wave does not overlap the
// matrix pipe (measured, tools/mfma_probe.hip: four 32x32x2 MFMAs per K*
// value run at 86 % of peak, sixteen 16x16x4 MFMAs per K* value at 91 %), so
// the K* chain (2 sub, mul, fma, mul, exp) must be amortised over as many
// MFMAs as the register file allows.  256 rows x 16 queries per wave is 64
// accumulator registers plus 64 (f32) or 128 (f64) for the cross-tile sum,
// which leaves two waves per SIMD.
//
// The A tile [BK = 64][BM = 256] is staged through LDS by LDS-DMA (double
// buffered, one barrier per stage).  tile_offset puts the four A operands of
// row blocks 4jj..4jj+3 of one (k, row&15) side by side, so a k step is four
// conflict-free ds_read_b128 per lane.  The mean rides along in the last row
// block (every kept k visited) as an f64 FMA per k step.
//
// Plan, then sweep.  plan_count_kernel decides, per work item, which k-tiles
// run (error-budgeted, see below) and counts them; a scan turns the counts
// into offsets; plan_write_kernel writes the kept tile indices (ascending)
// and a descriptor per non-empty item, in row-block-major order, heaviest
// row block first; plan_seg_kernel cuts that item list into one contiguous,
// tile-balanced range per workgroup.  predict_kernel is persistent (one
// workgroup per CU): it walks its range as one flat stream of (item, tile)
// steps, so the LDS-DMA pipeline runs across item boundaries, and neither
// the selection nor empty items nor workgroup launches cost sweep time
// (measured on a launch-per-item kernel: selection 5.9 %, empty items 3 %,
// launch gaps ~6 % of the C4 sweep).
//
// Tile selection: with the tile-norm table (automatic cutoff) each item
// bounds tile t's share of |dV_I(q)|_2 by nu_It * K*max(box distance) and
// drops tiles smallest bound first while the dropped bounds stay within the
// row block's budget (binned, fixed point: order-independent); otherwise a
// tile whose bounding box is farther from the query block's box than the
// cutoff radius (every K* < 2^-L) is dropped.  The last row block also keeps
// every tile within the mean's cutoff.  Kept tiles run in ascending t, the
// dense order, so L >= 150 (only exact zeros dropped) is bitwise identical
// to the dense sweep.
//
// Accuracy: a single f32 MFMA chain over all N training points accumulates
// ~sqrt(N) roundings on large cancelling terms (2.2e-5 normwise variance
// error at N = 8192, measured).  Each k-tile's chain therefore starts from
// zero and is added into an outer accumulator; the K* evaluation error
// (f32 coordinate differences and exp2), amplified by A, dominates what is
// left (tools/variant_accuracy.py: 5e-6 at N = 16384 for either outer type).
constexpr int kStageFloats = kTileFloats + 3 * kBK;
constexpr int kPredictWaves = kBN / 16;
constexpr int kPredictThreads = 64 * kPredictWaves;
constexpr int kDescWindow = 64;          // item descriptors (int4) per 1 KiB LDS window
constexpr int kListWindow = 512;         // tile indices (u16) per 1 KiB LDS window
constexpr int kRecWindow = 64;           // split-sweep step records (int4) per 1 KiB LDS window
constexpr int kSmemFloats = 2 * kStageFloats + 2 * 256 + 2 * 256;  // stages + 2 desc + 2 list windows
constexpr int kBudgetFloor = 40;        // bounds below 2^-40 of the budget share bin 0
constexpr int kBinsPerBit = 4;
constexpr int kBudgetBins = kBudgetFloor * kBinsPerBit + 2;
constexpr int kPlanThreads = 256;       // plan kernels: one query block, one row block per wave
constexpr int kPlanWaves = kPlanThreads / 64;
constexpr int kPlanD2 = 2048;           // k-tile distances cached in LDS (N <= 131072; beyond: recomputed)
constexpr int kPlanBinCache = 256;
constexpr int kPlanWriteBlocks = 4096;  // plan_write grid cap (four waves each, grid-stride over items)      // per wave: the increment bins of a row block's first tiles (nI <= 64: all)
constexpr int kPlanKeyShift = 40;       // plan key: kept-tile count (low 40 bits) | non-empty (high bits)
constexpr unsigned long long kPlanCountMask = (1ull << kPlanKeyShift) - 1ull;
// Sweep time of a kept tile by precision level, in 1/64 of a full tile
// (forced-level C4 sweeps: 20.6, 13.5, 10.6 ns per tile): the weight the
// workgroup ranges and sbo_query_cost balance
constexpr unsigned kLevelWeight0 = 64, kLevelWeight1 = 42, kLevelWeight2 = 33;
// The mean's row block (the last) sweeps slower per tile than the others --
// stamp build at C4 with every tile forced to one level: the XCD chunk that
// holds it balanced at 125 / 107 / 100 % of the six- / three- / one-product
// weights -- and lower row blocks somewhat faster (their A operand fits the
// XCD's L2): tile weights of the mean's row block, and the slope, percent at
// I = nI - 1 over I = 0, of a linear per-row-block factor (diagnostic build:
// SBO_MEAN_W = "w0,w1,w2", SBO_RB_SLOPE)
constexpr unsigned kMeanWeight0 = 80, kMeanWeight1 = 45, kMeanWeight2 = 33;
__device__ unsigned g_mean_w[3] = {kMeanWeight0, kMeanWeight1, kMeanWeight2};
__device__ unsigned g_rb_slope = 0;
constexpr int kSteps = kBK / 4;          // 16x16x4 k steps per tile
constexpr int kRowBlocks = kBM / 16;     // 16-row MFMA blocks per wave

typedef float f32x4 __attribute__((ext_vector_type(4)));

// The sixteen k steps of one staged tile: acc = A_tile * K*_tile (fresh
// chain), mean += sf2 alpha^T K* when MEAN.
//
// Software pipeline, pinned with scheduling fences (left alone, the compiler
// minimises registers by issuing each A read right before its MFMA and then
// waiting on it): step p first issues the LDS reads of the A operands of
// step p+1 (four ds_read_b128 = the sixteen row blocks, tile_offset layout);
// every even step also reads the coordinate pairs of steps p+4, p+5 and
// evaluates K* of steps p+2, p+3 as one packed pair (v_pk_add/mul/fma_f32,
// then two v_exp_f32) beside the sixteen MFMAs of step p.  No MFMA or exp
// waits on a read issued in its own step.  pc = this lane group's
// coordinate row (kcoord_slot layout: step p of x at pc[p], y at
// pc[kBK + p], sf2*alpha at pc[2*kBK + p]).
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x2 kstar_pair(f32x2 x, f32x2 y, float xq, float yq, float cexp) {
    const f32x2 dx = x - xq, dy = y - yq;
    const f32x2 d2 = __builtin_elementwise_fma(dy, dy, dx * dx);
    const f32x2 a = d2 * cexp;
    f32x2 b;
    b.x = fast_exp2(a.x);
    b.y = fast_exp2(a.y);
    return b;
}

template <bool MEAN>
__device__ __forceinline__ void tile_steps(const float4 *__restrict__ pa, const float *__restrict__ pc, float xq,
                                           float yq, float cexp, f32x4 (&acc)[kRowBlocks], double &mu) {
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
    const f32x2 *pc2 = reinterpret_cast<const f32x2 *>(pc);
    float4 a_cur[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) a_cur[jj] = pa[jj * 1024];
    f32x2 b_cur = kstar_pair(pc2[0], pc2[kBK / 2], xq, yq, cexp);  // steps 0, 1
    f32x2 x1 = pc2[1], y1 = pc2[kBK / 2 + 1];                         // steps 2, 3
    f32x2 b_nxt = b_cur;
#pragma unroll
    for (int p = 0; p < kSteps; ++p) {
        float4 a_nxt[4];
        f32x2 x2 = x1, y2 = y1;
        if (p + 1 < kSteps) {
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) a_nxt[jj] = pa[jj * 1024 + (p + 1) * 64];
        }
        if ((p & 1) == 0 && p + 4 < kSteps) {
            x2 = pc2[(p + 4) / 2];
            y2 = pc2[kBK / 2 + (p + 4) / 2];
        }
        const float alpha = MEAN ? pc[2 * kBK + p] : 0.0f;
        __builtin_amdgcn_sched_barrier(0);
        if ((p & 1) == 0 && p + 2 < kSteps) b_nxt = kstar_pair(x1, y1, xq, yq, cexp);
        const float b = (p & 1) ? b_cur.y : b_cur.x;
        if (MEAN) mu = fma((double)alpha, (double)b, mu);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            acc[4 * jj + 0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a_cur[jj].x, b, p == 0 ? zero : acc[4 * jj + 0], 0, 0, 0);
            acc[4 * jj + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a_cur[jj].y, b, p == 0 ? zero : acc[4 * jj + 1], 0, 0, 0);
            acc[4 * jj + 2] = __builtin_amdgcn_mfma_f32_16x16x4f32(a_cur[jj].z, b, p == 0 ? zero : acc[4 * jj + 2], 0, 0, 0);
            acc[4 * jj + 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a_cur[jj].w, b, p == 0 ? zero : acc[4 * jj + 3], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (p + 1 < kSteps) {
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) a_cur[jj] = a_nxt[jj];
        }
        if ((p & 1) == 0) {
            x1 = x2;
            y1 = y2;
        } else {
            b_cur = b_nxt;
        }
    }
}

__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fminf(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}

// ---- plan: which k-tiles each work item (I, qb) multiplies
struct QBox {
    float x0, x1, y0, y1;
};

__device__ __forceinline__ float tile_box_d2(const float4 b, const QBox &q) {
    // b = (xmin, xmax, ymin, ymax); an empty tile (+inf, -inf, ..) is infinitely far
    const float dx = fmaxf(0.0f, fmaxf(b.x - q.x1, q.x0 - b.y));
    const float dy = fmaxf(0.0f, fmaxf(b.z - q.y1, q.y0 - b.w));
    return fmaf(dy, dy, dx * dx);
}

// A kept tile runs at one of three precision levels: all six split
// products (code 0), the three largest a1 k0 + a0 k1 + a0 k0 (code 1), or
// a0 k0 alone (code 2).  With A = A0 + A1 + A2 and K = K0 + K1 + K2 the
// bf16 pieces (round to nearest at each step, so |K1| <= 2^-9 (1 + 2^-9) |K|
// and |K2| <= 2^-18 (1 + 2^-9)^2 |K| entrywise), the products code 1 leaves
// out are A2 K0 + A1 K1 + A0 K2 and code 2 also A1 K0 + A0 K1; each is
// bounded plane by plane, |A_p K_j|_2 <= min(R_p K*max, S_p |k|_2) rho_j with
// R_p = 16 max row 1-norm and S_p the spectral bound of piece p (lgn[2T+1];
// for A0: R = R_A (1 + 2^-9), S = S_A + 2^-9 |A|_F).  Lowering a tile's
// level, or dropping it, costs part of the row block's error budget; the
// three increments
//     code 0 -> 1:  c3 = |A2 K0| + |A1 K1| + |A0 K2|   (bounds as above)
//     code 1 -> 2:  c1 = |A1 K0| + |A0 K1|
//     code 2 -> drop:  b - c3 - c1,  b = min(R_A K*max, S_A |k|_2) >= |A_It k_t|_2
// sum to the tile's drop bound and are spent greedily over all tiles of the
// row block, cheapest first by error per sweep time saved (the increments
// are ranked by log2(error) + kLvlKey[j], kLvlKey from the measured per-tile
// time of the three levels and of the drop; a tile's keys never go down, so
// its spent increments are a prefix).  (Earlier rule, still an upper bound
// of these: c3 <= 3.1 2^-16 |A|_F |k|_2, c3 + c1 <= 2.03 2^-8 |A|_F |k|_2 --
// far_tile relies on it.)
// For each increment: its bin relative to the budget 2^lg_tau (bin 0 = below
// 2^-kBudgetFloor of it, bin kBudgetBins-1 = over the whole budget, never
// spent) and its weight in fixed point (2^32 = the budget), rounded up.
constexpr float kLg3 = -14.36f;  // log2(3.1 2^-16), rounded up
constexpr float kLg1 = -6.96f;   // log2(2.03 2^-8 + 3.1 2^-16), rounded up
constexpr float kRho0 = 0.0029f;          // log2(1 + 2^-9), rounded up
constexpr float kRho1 = -9.0f + 0.0029f;  // log2(2^-9 (1 + 2^-9))
constexpr float kRho2 = -18.0f + 0.0058f; // log2(2^-18 (1 + 2^-9)^2)

__device__ __forceinline__ int inc_bin(float l, unsigned long long &w, float key = 0.0f) {  // l = log2(inc / budget)
    const float f = (l + key + (float)kBudgetFloor) * (float)kBinsPerBit + 1.0f;
    const int bi = f < 0.0f ? 0 : (f >= (float)(kBudgetBins - 1) ? kBudgetBins - 1 : (int)f);
    w = bi < kBudgetBins - 1 ? (unsigned long long)ceilf(exp2f(l + 32.0f) * 1.0001f) + 1ull : 0ull;
    return bi;
}

// log2(2^a + 2^b), rounded up
__device__ __forceinline__ float lg_add(float a, float b) {
    const float hi = fmaxf(a, b), lo = fminf(a, b);
    return hi + __log2f(1.0f + exp2f(lo - hi)) + 1e-4f;
}

__device__ __forceinline__ void tile_increments(float d2, float kn, float4 lgn_t, float4 lgp_t, float cexp,
                                                float lg_tau, float2 key, int (&bi)[3],
                                                unsigned long long (&w)[3]) {
    const float kmax = cexp * d2 * 0.999f;
    const float b = fminf(lgn_t.x + kmax, lgn_t.y + kn) - lg_tau + 0.01f;
    // |A_p k|_2 bounds of the three pieces (relative to the budget)
    const float n0 = fminf(lgn_t.x + kRho0 + kmax, lg_add(lgn_t.y, lgn_t.z - 9.0f) + kn) - lg_tau + 0.01f;
    const float n1 = fminf(lgp_t.x + kmax, lgp_t.y + kn) - lg_tau + 0.01f;
    const float n2 = fminf(lgp_t.z + kmax, lgp_t.w + kn) - lg_tau + 0.01f;
    const float r3 = lg_add(lg_add(n2 + kRho0, n1 + kRho1), n0 + kRho2);   // A2 K0 + A1 K1 + A0 K2
    const float r1 = lg_add(n1 + kRho0, n0 + kRho1);                       // A1 K0 + A0 K1
    const float r31 = lg_add(r3, r1);
    bi[0] = inc_bin(r3, w[0], key.x);
    bi[1] = inc_bin(r1, w[1], key.y);
    const float dl = r31 - b;
    bi[2] = dl < -0.01f ? inc_bin(b + __log2f(1.0f - exp2f(dl)), w[2]) : inc_bin(b, w[2]);
    // monotone: the three bins never go down (so a tile's spent increments are a prefix)
    bi[1] = max(bi[1], bi[0]);
    bi[2] = max(bi[2], bi[1]);
}

// Everything the two plan kernels share: the query block's box, the box
// distance of every k-tile, and the per-item selection rule.
struct PlanRule {
    const float4 *kbox;
    const float4 *lgn;  // per packed tile log2 gain bounds, two float4 (null: distance test)
    float cexp, skip_d2, skip_d2_mean, lg_tau;
    int nI;
    QBox box;
    const float *d2s;   // LDS cache of tile distances (t < kPlanD2)
    const float *kns;   // LDS cache of the tiles' log2 |k|_2 bounds (t < kPlanD2)
    int levels;         // 0: every kept tile at full precision; 1: budgeted levels; 2 + l: timing
                        // diagnostic, the drop-only plan with every kept tile at level l
    float2 key;         // rank keys of the two level increments (SkipPlan::lvl_key)

    __device__ __forceinline__ float d2(int t) const { return t < kPlanD2 ? d2s[t] : tile_box_d2(kbox[t], box); }
    // beyond the cache: |k|_2 <= 8 K*max
    __device__ __forceinline__ float kn(int t) const { return t < kPlanD2 ? kns[t] : 3.0f + cexp * d2(t) * 0.999f; }

    // A tile whose largest possible increment (the drop bound by K*max, plus
    // the larger level rank key) is below bin 0's upper edge: all three of
    // its increments go to bin 0 with weight <= 2 each (exp2(l + 32) < 2^-8
    // rounds up to at most 1, plus 1), so the plan books 6 for it without
    // evaluating the bounds -- most candidate tiles of a row block.
    __device__ __forceinline__ bool far_tile(int I, int t, float dd) const {
        const float kf = fmaxf(0.0f, fmaxf(key.x + kLg3, key.y + kLg1));
        return lgn[2 * (tile_start(I) + t)].x + cexp * dd * 0.999f - lg_tau + 0.01f + kf < -(float)kBudgetFloor;
    }

    __device__ __forceinline__ void incs(int I, int t, int (&bi)[3], unsigned long long (&w)[3]) const {
        const int64_t T = tile_start(I) + t;
        tile_increments(d2(t), kn(t), lgn[2 * T], lgn[2 * T + 1], cexp, lg_tau, key, bi, w);
        if (levels != 1) {  // only the whole drop: the first two increments free, the third the whole drop bound
            bi[0] = bi[1] = 0;
            w[0] = w[1] = 0ull;
            const float kmax = cexp * d2(t) * 0.999f;
            const float4 l = lgn[2 * T];
            bi[2] = inc_bin(fminf(l.x + kmax, l.y + kn(t)) - lg_tau + 0.01f, w[2]);
        }
    }

    // Total weight of every increment of row block I (wave-wide): what the
    // row block would spend dropping all its tiles; `over` is set when some
    // increment is larger than the whole reference budget (it never drops
    // everything).  The same increments and fixed-point weights as threshold.
    __device__ unsigned long long total_weight(int I, int lane, bool &over) const {
        const int T = kTilesPerRowBlockStep * (I + 1);
        unsigned long long wsum = 0;
        int ov = 0;
        for (int t0 = 0; t0 < T; t0 += 64) {
            const int t = t0 + lane;
            if (t < T) {
                if (far_tile(I, t, d2(t))) {
                    wsum += 6ull;
                } else {
                    int bi[3];
                    unsigned long long w[3];
                    incs(I, t, bi, w);
#pragma unroll
                    for (int j = 0; j < 3; ++j) {
                        if (bi[j] < kBudgetBins - 1) wsum += w[j];
                        else ov = 1;
                    }
                }
            }
            // an increment over the whole budget decides the row block (never
            // cheap): the rest of its tiles cannot change that
            if (__ballot(ov)) break;
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            wsum += __shfl_xor(wsum, o);
            ov |= __shfl_xor(ov, o);
        }
        over = ov != 0;
        return wsum;
    }

    // Greedy budget threshold of row block I (wave-wide; bins is wave-private
    // LDS): the largest prefix of bins, smallest increments first, whose
    // summed weights (integer adds: order-independent) stay within the
    // row block's budget (fixed point, 2^32 = the reference budget 2^lg_tau).
    // Returns the last spent bin (-1: none).
    __device__ int threshold(int I, unsigned long long *bins, int lane, unsigned long long budget,
                             unsigned *bc = nullptr) const {
        if (!lgn) return -1;
        const int T = kTilesPerRowBlockStep * (I + 1);
        for (int i = lane; i < kBudgetBins; i += 64) bins[i] = 0ull;
        __builtin_amdgcn_wave_barrier();
        unsigned long long nfar = 0;
        for (int t = lane; t < T; t += 64) {
            if (far_tile(I, t, d2(t))) {
                ++nfar;
                if (bc && t < kPlanBinCache) bc[t] = 0u;  // all three increments in bin 0
                continue;
            }
            int bi[3];
            unsigned long long w[3];
            incs(I, t, bi, w);
            if (bc && t < kPlanBinCache) bc[t] = (unsigned)bi[0] | ((unsigned)bi[1] << 8) | ((unsigned)bi[2] << 16);
#pragma unroll
            for (int j = 0; j < 3; ++j)
                if (bi[j] < kBudgetBins - 1) atomicAdd(bins + bi[j], w[j]);
        }
        if (nfar) atomicAdd(bins, 6ull * nfar);
        __builtin_amdgcn_wave_barrier();
        constexpr int per = (kBudgetBins + 63) / 64;
        unsigned long long v[per], run = 0;
#pragma unroll
        for (int j = 0; j < per; ++j) {
            const int i = lane * per + j;
            v[j] = i < kBudgetBins - 1 ? bins[i] : (1ull << 40);
            run += v[j];
        }
        unsigned long long incl = run;  // inclusive scan over lanes
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned long long u = __shfl_up(incl, o);
            if (lane >= o) incl += u;
        }
        unsigned long long pre = incl - run;
        int ok = 0;
#pragma unroll
        for (int j = 0; j < per; ++j) {
            pre += v[j];
            ok += pre <= budget ? 1 : 0;
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) ok += __shfl_xor(ok, o);
        __builtin_amdgcn_wave_barrier();
        return ok - 1;
    }

    // The tile's level code (0 full, 1 three products, 2 one product) or -1
    // (dropped) under the row block's threshold.  bc: the bins threshold()
    // cached for this row block (a far tile's are all 0, as booked there).
    __device__ __forceinline__ int level(int I, int t, int drop_max, const unsigned *bc = nullptr) const {
        const float dd = d2(t);
        int code;
        if (lgn) {
            int spent;
            if (bc && t < kPlanBinCache) {
                const unsigned c = bc[t];
                spent = ((int)(c & 0xffu) <= drop_max) + ((int)((c >> 8) & 0xffu) <= drop_max) +
                        ((int)(c >> 16) <= drop_max);
            } else if (far_tile(I, t, dd)) {
                spent = drop_max >= 0 ? 3 : 0;
            } else {
                int bi[3];
                unsigned long long w[3];
                incs(I, t, bi, w);
                spent = (bi[0] <= drop_max) + (bi[1] <= drop_max) + (bi[2] <= drop_max);
            }
            code = spent == 3 ? -1 : (levels == 1 ? spent : (levels > 1 ? levels - 2 : 0));
        } else {
            code = (skip_d2 <= 0.0f || dd <= skip_d2) ? 0 : -1;  // skip_d2 <= 0: dense
        }
        // the mean's own cutoff (last row block): keep at the cheapest level
        // (its V error is below the drop bound already spent)
        if (code < 0 && I == nI - 1 && dd <= skip_d2_mean) code = lgn && levels ? 2 : 0;
        return code;
    }
};

// The plan's reference budget 2^lg_ref = tau2, the whole query block's
// |dV|_2 budget, from lg_tau = log2(tau2 / sqrt(nI)) (the even share).
__device__ __forceinline__ float plan_ref(float lg_tau, int nI) { return lg_tau + 0.5f * __log2f((float)nI) - 1e-4f; }
constexpr int kPlanMaxI = 512;   // water-filling of the budget for nI <= this (N <= 131072), else even shares

// Query box of block qb (threads 0..127 hold its queries, 128..255 repeat
// them) and the distance cache.
// Bound on log2 |k_t(q)|_2 for every query q of the box: the tile's points p
// (kcoord; padding points count too, which only raises the bound) give
// K*(p, q) <= 2^(cexp dist(p, box)^2), so |k|_2^2 <= sum_p 2^(2 cexp dist^2)
// (summed scaled by 2^120 against underflow; 0.999 / 1.002 margins over the
// kernel's f32 rounding); if even that underflows, the box bound 8 K*max.
__device__ __forceinline__ float tile_knorm(const float *__restrict__ kc, const QBox &b, float cexp, float d2box) {
    float sum = 0.0f;
    for (int i = 0; i < kBK; ++i) {
        const float px = kc[i], py = kc[kBK + i];
        const float dx = fmaxf(0.0f, fmaxf(b.x0 - px, px - b.x1));
        const float dy = fmaxf(0.0f, fmaxf(b.y0 - py, py - b.y1));
        sum += __builtin_amdgcn_exp2f(fmaf(2.0f * cexp, fmaf(dy, dy, dx * dx) * 0.999f, 120.0f));
    }
    return sum > 0.0f ? 0.5f * (__log2f(sum * 1.002f) - 120.0f) + 0.001f : 3.0f + cexp * d2box * 0.999f;
}

__device__ QBox plan_setup(const float *__restrict__ qx, const float *__restrict__ qy, int64_t m, int64_t qb,
                           const float4 *__restrict__ kbox, const float *__restrict__ kcoord, float cexp, int nkt,
                           float *d2s, float *kns, float *red) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t q = qb * kBN + (tid & (kBN - 1));
    const int64_t qc = q < m ? q : m - 1;
    const float xq = qx[qc], yq = qy[qc];
    const float bx0 = wave_min(xq), bx1 = wave_max(xq), by0 = wave_min(yq), by1 = wave_max(yq);
    if (lane == 0) {
        red[wave * 4 + 0] = bx0; red[wave * 4 + 1] = bx1;
        red[wave * 4 + 2] = by0; red[wave * 4 + 3] = by1;
    }
    __syncthreads();
    QBox b = {red[0], red[1], red[2], red[3]};
#pragma unroll
    for (int w = 1; w < kPlanWaves; ++w) {
        b.x0 = fminf(b.x0, red[w * 4 + 0]); b.x1 = fmaxf(b.x1, red[w * 4 + 1]);
        b.y0 = fminf(b.y0, red[w * 4 + 2]); b.y1 = fmaxf(b.y1, red[w * 4 + 3]);
    }
    for (int t = tid; t < nkt && t < kPlanD2; t += kPlanThreads) {
        const float d = tile_box_d2(kbox[t], b);
        d2s[t] = d;
        // only tiles whose box bound can reach the budget floors need the point sum
        kns[t] = (kcoord && cexp * d > -400.0f) ? tile_knorm(kcoord + (int64_t)t * (3 * kBK), b, cexp, d)
                                                : 3.0f + cexp * d * 0.999f;
    }
    __syncthreads();
    return b;
}

// Item index of (I, qb): row-block major, heaviest (last) row block first.
// Item order (round 5): row-block-major, heaviest row block first; with
// blk = bi << 8 | bq (> 0, the precise sweep's SBO_OPT_PLAN_BLOCK) in blocks
// of bi row blocks x bq query blocks, so that the sweep workgroups of one XCD,
// which run consecutive items at once, share the K* table pieces of a query
// block (bi of them) as well as the A tiles of a row block (bq of them) in
// their L2 -- instead of 32-fold A sharing and no table sharing.  A bijection
// of [0, nI nQ); plan_item_inv inverts it.
__device__ __forceinline__ int64_t plan_item(int I, int nI, int64_t nQ, int64_t qb, int blk = 0) {
    const int64_t r = nI - 1 - I;
    if (blk == 0) return r * nQ + qb;
    const int64_t bi = blk >> 8, bq = blk & 255;
    const int64_t IB = r / bi, ii = r % bi, QB = qb / bq, qq = qb % bq;
    const int64_t bie = min(bi, (int64_t)nI - IB * bi), bqe = min(bq, nQ - QB * bq);
    return IB * bi * nQ + QB * bie * bq + ii * bqe + qq;
}
__device__ __forceinline__ void plan_item_inv(int64_t item, int nI, int64_t nQ, int blk, int &I, int64_t &qb) {
    if (blk == 0) {
        I = nI - 1 - (int)(item / nQ);
        qb = item % nQ;
        return;
    }
    const int64_t bi = blk >> 8, bq = blk & 255;
    const int64_t IB = item / (bi * nQ), r0 = item - IB * bi * nQ;
    const int64_t bie = min(bi, (int64_t)nI - IB * bi);
    const int64_t QB = r0 / (bie * bq), r1 = r0 - QB * bie * bq;
    const int64_t bqe = min(bq, nQ - QB * bq);
    I = nI - 1 - (int)(IB * bi + r1 / bqe);
    qb = QB * bq + r1 % bqe;
}
// 64-tile chunks of the longest item (the code bitmap's stride per item)
__host__ __device__ __forceinline__ int plan_chunks(int nI) { return (kTilesPerRowBlockStep * nI + 63) / 64; }

// Pass 1, one workgroup per query block, one row block per wave at a time:
// the budget threshold and the kept-tile count of every item.  key packs
// (count, non-empty) for the scan; empty items get their (exactly zero)
// outputs here, so the sweep never visits them.
__global__ __launch_bounds__(kPlanThreads) void plan_count_kernel(
    const float4 *__restrict__ kbox, const float *__restrict__ kcoord, const float4 *__restrict__ lgn, int levels,
    float2 lvl_key, int nI,
    int64_t nQ,
    const float *__restrict__ qx, const float *__restrict__ qy, int64_t m, float cexp, float skip_d2,
    float skip_d2_mean, float lg_tau, float m0, int64_t ldp, float *__restrict__ part, float *__restrict__ mean,
    unsigned long long *__restrict__ key, unsigned char *__restrict__ thr, unsigned long long *__restrict__ wkey,
    unsigned long long *__restrict__ bits, int wide, int blk) {
    // dynamic LDS: the increment-bin cache [kPlanWaves][kPlanBinCache], then
    // the distance and |k|_2 caches of min(nkt, kPlanD2) tiles each
    extern __shared__ unsigned plan_dyn[];
    __shared__ float red[4 * kPlanWaves];
    __shared__ unsigned long long bins[kPlanWaves][kBudgetBins];
    __shared__ unsigned long long wtot[kPlanMaxI];
    __shared__ unsigned long long budget_exp;
    const int64_t qb = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nkt = kTilesPerRowBlockStep * nI;
    unsigned *bc = plan_dyn + wave * kPlanBinCache;
    float *d2s = reinterpret_cast<float *>(plan_dyn + kPlanWaves * kPlanBinCache);
    float *kns = d2s + min(nkt, kPlanD2);
    PlanRule R{kbox, lgn, cexp, skip_d2, skip_d2_mean, plan_ref(lg_tau, nI), nI, {}, d2s, kns, levels, lvl_key};
    R.box = plan_setup(qx, qy, m, qb, kbox, lgn ? kcoord : nullptr, cexp, nkt, d2s, kns, red);
    // The error budget of the query block, |dV(q)|_2^2 = sum_I |dV_I(q)|_2^2
    // <= tau2^2 = 2^(2 lg_ref) for every query q of the block, shared over
    // its row blocks by water-filling instead of evenly (tau2 / sqrt(nI)
    // each): a row block whose tiles can all be dropped within the common
    // share drops them and spends only what they cost; the rest of tau2^2 is
    // split evenly over the others (iterated: a larger share can make more
    // row blocks cheap).  Fixed point, 2^32 = 2^lg_ref.
    const bool fill = lgn && nI <= kPlanMaxI;
    if (fill) {
        for (int I = wave; I < nI; I += kPlanWaves) {
            bool over;
            const unsigned long long w = R.total_weight(I, lane, over);
            if (lane == 0) wtot[I] = over ? ~0ull : w;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            const double one = 4294967296.0;
            double share = 1.0 / sqrt((double)nI);   // the even split, in units of 2^lg_ref
            for (int it = 0; it < 4; ++it) {
                double cheap2 = 0.0;
                int nexp = 0;
                for (int I = 0; I < nI; ++I) {
                    const double w = wtot[I] == ~0ull ? 2.0 : (double)wtot[I] / one;
                    if (w <= share) cheap2 += w * w;
                    else ++nexp;
                }
                if (nexp == 0) break;
                const double s2 = fmax(0.0, (1.0 - cheap2) * (1.0 - 1e-9)) / (double)nexp;
                const double sn = sqrt(s2) * (1.0 - 1e-9);
                if (!(sn > share)) break;
                share = sn;
            }
            budget_exp = (unsigned long long)floor(share * one);
        }
        __syncthreads();
    }
    for (int I = wave; I < nI; I += kPlanWaves) {
        const int T = kTilesPerRowBlockStep * (I + 1);
        // a cheap row block (everything within the share) spends its own total
        const unsigned long long bud = !fill ? (unsigned long long)floor(4294967296.0 / sqrt((double)nI))
                                       : (wtot[I] <= budget_exp ? ~0ull : budget_exp);
        const int drop_max = R.threshold(I, bins[wave], lane, bud, bc);
        const int64_t item = plan_item(I, nI, nQ, qb, blk);
        // the item's codes, 64 tiles per chunk: kept / level 1 / level 2 masks (read by plan_write)
        unsigned long long *ib = bits + item * (int64_t)plan_chunks(nI) * 3;
        int cnt = 0;
        unsigned wsum = 0;
#pragma unroll 1
        for (int t0 = 0; t0 < T; t0 += 64) {
            const int t = t0 + lane;
            const int code = t < T ? R.level(I, t, drop_max, bc) : -1;
            const unsigned long long b0 = __ballot(code == 0), b1 = __ballot(code == 1), b2 = __ballot(code == 2);
            if (lane < 3) ib[(t0 >> 6) * 3 + lane] = lane == 0 ? (b0 | b1 | b2) : (lane == 1 ? b1 : b2);
            const int n0 = __popcll(b0), n1 = __popcll(b1), n2 = __popcll(b2);
            cnt += n0 + n1 + n2;
            wsum += I == nI - 1 ? g_mean_w[0] * n0 + g_mean_w[1] * n1 + g_mean_w[2] * n2
                                : kLevelWeight0 * n0 + kLevelWeight1 * n1 + kLevelWeight2 * n2;
        }
        if (g_rb_slope)
            wsum = (unsigned)((unsigned long long)wsum * (100u * (unsigned)nI + g_rb_slope * (unsigned)I) /
                              (100u * (unsigned)nI));
        if (lane == 0) {
            key[item] = (unsigned long long)cnt | ((cnt > 0 ? 1ull : 0ull) << kPlanKeyShift);
            thr[item] = (unsigned char)(drop_max + 1);
            wkey[item] = wsum;
        }
        if (cnt == 0)
            for (int j = lane; j < kBN; j += 64) {
                const int64_t q = qb * kBN + j;
                if (q < m) {
                    // (wide: the precise sweep's f64 partials and mean)
                    if (wide) {
                        reinterpret_cast<double *>(part)[(int64_t)I * ldp + q] = 0.0;
                        if (I == nI - 1) reinterpret_cast<double *>(mean)[q] = (double)m0;
                    } else {
                        part[(int64_t)I * ldp + q] = 0.0f;
                        if (I == nI - 1) mean[q] = m0;
                    }
                }
            }
    }
}

// Pass 2 (after the inclusive scan of key): the kept tile indices of every
// non-empty item, ascending, at its offset, and its descriptor
// (I, qb, offset low 32 bits, count | offset high bits << 16) -- from the
// code bitmap plan_count left (bits: per item and 64-tile chunk, the kept /
// level-1 / level-2 masks), so no tile's bounds are evaluated twice.  Each
// wave walks items gw, gw + W, .. (W = all waves of the grid).
__global__ __launch_bounds__(256) void plan_write_kernel(
    int nI, int64_t nQ, const unsigned long long *__restrict__ key, const unsigned long long *__restrict__ scan,
    const unsigned long long *__restrict__ bits, int4 *__restrict__ desc, unsigned short *__restrict__ tl,
    int prod_full, unsigned long long *__restrict__ partial, int blk) {
    // partial (may be null): per wave [MFMA products, tiles at level 1, at level 2]
    // (summed by plan_counts_reduce_kernel: no contended global atomics)
    const int lane = threadIdx.x & 63;
    const int64_t gw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (int64_t)gridDim.x * 4;
    const int64_t items = (int64_t)nI * nQ;
    unsigned long long prod = 0, nl1 = 0, nl2 = 0;
    for (int64_t item = gw; item < items; item += nw) {
        const unsigned long long k = key[item];
        const int cnt = (int)(k & kPlanCountMask);
        if (cnt > 0) {
            int I;
            int64_t qb;
            plan_item_inv(item, nI, nQ, blk, I, qb);
            const unsigned long long ex = scan[item] - k;
            const uint64_t off = ex & kPlanCountMask;
            const int64_t ne = (int64_t)(ex >> kPlanKeyShift);
            const int T = kTilesPerRowBlockStep * (I + 1);
            const unsigned long long *ib = bits + item * (int64_t)plan_chunks(nI) * 3;
            uint64_t base = off;
            for (int t0 = 0; t0 < T; t0 += 64) {
                const unsigned long long kept = ib[(t0 >> 6) * 3], l1 = ib[(t0 >> 6) * 3 + 1],
                                         l2 = ib[(t0 >> 6) * 3 + 2];
                if ((kept >> lane) & 1ull) {
                    const int code = ((l1 >> lane) & 1ull) ? 1 : (((l2 >> lane) & 1ull) ? 2 : 0);
                    tl[base + __popcll(kept & ((1ull << lane) - 1ull))] =
                        (unsigned short)((t0 + lane) | (code << kLevelShift));
                    prod += code == 0 ? prod_full : (code == 1 ? 3 : 1);
                    nl1 += code == 1 ? 1 : 0;
                    nl2 += code == 2 ? 1 : 0;
                }
                base += __popcll(kept);
            }
            if (lane == 0) desc[ne] = make_int4(I, (int)qb, (int)(uint32_t)off, cnt | (int)((off >> 32) << 16));
        }
    }
    if (partial) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            prod += __shfl_xor(prod, o);
            nl1 += __shfl_xor(nl1, o);
            nl2 += __shfl_xor(nl2, o);
        }
        if (lane == 0) {
            unsigned long long *p = partial + 3 * gw;
            p[0] = prod;
            p[1] = nl1;
            p[2] = nl2;
        }
    }
}

// One workgroup: the per-wave level counts of plan_write into the profile counters.
__global__ __launch_bounds__(256) void plan_counts_reduce_kernel(const unsigned long long *__restrict__ partial,
                                                                 int64_t n, unsigned long long *__restrict__ out) {
    __shared__ unsigned long long red[3][256];
    unsigned long long v[3] = {0, 0, 0};
    for (int64_t i = threadIdx.x; i < n; i += 256)
#pragma unroll
        for (int j = 0; j < 3; ++j) v[j] += partial[3 * i + j];
#pragma unroll
    for (int j = 0; j < 3; ++j) red[j][threadIdx.x] = v[j];
    __syncthreads();
    for (int o = 128; o >= 1; o >>= 1) {
        if ((int)threadIdx.x < o)
#pragma unroll
            for (int j = 0; j < 3; ++j) red[j][threadIdx.x] += red[j][threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0)
#pragma unroll
        for (int j = 0; j < 3; ++j) out[j] += red[j][0];
}

// One thread per sweep workgroup: cut the non-empty item list into P
// contiguous ranges of about equal sweep time -- the level-weighted tile
// count (wkey, inclusive scan wscan) -- (seg[r] .. seg[r+1]).
__global__ void plan_seg_kernel(const unsigned long long *__restrict__ scan, int64_t n_items,
                                const int4 *__restrict__ desc, int P, int *__restrict__ seg,
                                unsigned long long *__restrict__ tiles_done, const unsigned long long *__restrict__ wkey,
                                const unsigned long long *__restrict__ wscan, int nI, int64_t nQ, int blk) {
    const unsigned long long last = scan[n_items - 1];
    const uint64_t total = last & kPlanCountMask;
    const uint64_t wtotal = wscan[n_items - 1];
    const int64_t nne = (int64_t)(last >> kPlanKeyShift);
    for (int w = threadIdx.x; w <= P; w += blockDim.x) {
        if (w == P) {
            seg[P] = (int)nne;
            continue;
        }
        const uint64_t target = wtotal * (uint64_t)w / (uint64_t)P;
        int64_t lo = 0, hi = nne;  // first item whose weighted offset >= target
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            const int4 d = desc[mid];
            const int64_t it = plan_item(d.x, nI, nQ, d.y, blk);
            const uint64_t off = wscan[it] - wkey[it];
            if (off < target) lo = mid + 1; else hi = mid;
        }
        seg[w] = (int)lo;
    }
    if (threadIdx.x == 0 && tiles_done) atomicAdd(tiles_done, (unsigned long long)total);
}

// XCD-interleaved item order (P a multiple of 8).  The sweep's workgroup b
// runs on XCD b % 8, and an XCD's 32 CUs share one L2: with contiguous
// per-workgroup ranges they work on 32 far-apart items at once and share no
// A tile (the staged bytes all come from beyond L2).  Instead each XCD takes
// one tile-balanced contiguous chunk [a, b) of the item list (plan_seg with
// 8 ranges, xseg), and its G = P/8 workgroups take the chunk's items
// round-robin -- slot c runs items a + c, a + c + G, ... -- so at any time
// they sweep G neighbouring items (same row block, Morton-adjacent query
// blocks, mostly the same k-tiles).  The descriptors and tile lists are
// permuted so that every workgroup's items stay contiguous (the sweep walks
// one contiguous range either way).
__device__ __forceinline__ int64_t xcd_position(int64_t k, const int *__restrict__ xseg, int G) {
    int x = 0;
#pragma unroll
    for (int i = 1; i < 8; ++i) x += k >= xseg[i] ? 1 : 0;
    const int64_t a = xseg[x], n = xseg[x + 1] - a, q = n / G, rm = n % G, c = (k - a) % G, j = (k - a) / G;
    return a + c * q + (c < rm ? c : rm) + j;
}

__global__ void plan_perm_kernel(const unsigned long long *__restrict__ scan, int64_t n_items,
                                 const int4 *__restrict__ desc, const int *__restrict__ xseg, int G,
                                 int *__restrict__ pos_of, unsigned long long *__restrict__ cnt2) {
    const int64_t nne = (int64_t)(scan[n_items - 1] >> kPlanKeyShift);
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nne) return;
    const int64_t p = xcd_position(k, xseg, G);
    pos_of[k] = (int)p;
    cnt2[p] = (unsigned long long)(desc[k].w & 0xffff);
}

__device__ __forceinline__ int4 step_record(int64_t ts, int I, int qb, int te, int i, int cnt);

// one wave per item: its tile list to the new offset, its descriptor to its
// new position, and (rec != nullptr) the split sweep's step records of the
// moved list -- what plan_rec_kernel would write from desc2 / tl2
__global__ __launch_bounds__(256) void plan_move_kernel(const unsigned long long *__restrict__ scan, int64_t n_items,
                                                        const int4 *__restrict__ desc,
                                                        const unsigned short *__restrict__ tl,
                                                        const int *__restrict__ pos_of,
                                                        const unsigned long long *__restrict__ off2,
                                                        int4 *__restrict__ desc2, unsigned short *__restrict__ tl2,
                                                        int4 *__restrict__ rec) {
    const int64_t nne = (int64_t)(scan[n_items - 1] >> kPlanKeyShift);
    const int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (k >= nne) return;
    const int4 d = desc[k];
    const int cnt = d.w & 0xffff;
    const uint64_t off = (uint64_t)(uint32_t)d.z | ((uint64_t)((uint32_t)d.w >> 16) << 32);
    const int p = pos_of[k];
    const uint64_t o2 = off2[p];
    const int64_t ts = tile_start(d.x);
    for (int i = lane; i < cnt; i += 64) {
        const unsigned short te = tl[off + i];
        tl2[o2 + i] = te;
        if (rec) rec[o2 + i] = step_record(ts, d.x, d.y, te, i, cnt);
    }
    if (lane == 0) desc2[p] = make_int4(d.x, d.y, (int)(uint32_t)o2, cnt | (int)((o2 >> 32) << 16));
}

// Step records of the split sweep (kRecFirst in sbo_internal.hpp), one
// wave per non-empty item, in the order the sweep walks the list (after the
// XCD permutation, where plan_move_kernel writes them): the kernel then
// stages a tile from one record instead of re-deriving offsets from the
// descriptor and tile list in every wave.
__device__ __forceinline__ int4 step_record(int64_t ts, int I, int qb, int te, int i, int cnt) {
    const int t = te & ((1 << kLevelShift) - 1);
    const int w = I | ((te >> kLevelShift) << 16) | (i == 0 ? kRecFirst : 0) | (i == cnt - 1 ? kRecLast : 0);
    return make_int4((int)(uint32_t)((ts + t) * 96), t * 256, qb, w);
}

__global__ __launch_bounds__(256) void plan_rec_kernel(const unsigned long long *__restrict__ scan, int64_t n_items,
                                                       const int4 *__restrict__ desc,
                                                       const unsigned short *__restrict__ tl, int4 *__restrict__ rec) {
    const int64_t nne = (int64_t)(scan[n_items - 1] >> kPlanKeyShift);
    const int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (k >= nne) return;
    const int4 d = desc[k];
    const int cnt = d.w & 0xffff;
    const uint64_t off = (uint64_t)(uint32_t)d.z | ((uint64_t)((uint32_t)d.w >> 16) << 32);
    const int64_t ts = tile_start(d.x);
    for (int i = lane; i < cnt; i += 64) rec[off + i] = step_record(ts, d.x, d.y, tl[off + i], i, cnt);
}

__global__ void plan_seg2_kernel(const int *__restrict__ xseg, int G, int P, int *__restrict__ seg2) {
    for (int r = threadIdx.x; r <= P; r += blockDim.x) {
        if (r == P) {
            seg2[P] = xseg[8];
            continue;
        }
        const int x = r / G, c = r % G;
        const int a = xseg[x], n = xseg[x + 1] - a, q = n / G, rm = n % G;
        seg2[r] = a + c * q + (c < rm ? c : rm);
    }
}

// Sweep work per query from a plan (load balancing across ranks): the kept
// tiles of its 128-query block summed over row blocks, shared by the block's
// queries; written in the caller's order (perm: sweep position -> caller).
__global__ void plan_block_cost_kernel(const unsigned long long *__restrict__ wkey, int nI, int64_t nQ,
                                       float *__restrict__ bcost) {
    const int64_t qb = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (qb >= nQ) return;
    unsigned long long c = 0;
    for (int I = 0; I < nI; ++I) c += wkey[plan_item(I, nI, nQ, qb)];
    bcost[qb] = (float)((double)c / (double)kLevelWeight0);  // in full-precision tiles
}

// a block's cost is shared by its queries (a grid patch's padded positions,
// perm -1, take no share): one block per workgroup of kBN threads
__global__ __launch_bounds__(kBN) void plan_query_cost_kernel(const float *__restrict__ bcost, int64_t m,
                                                              const int32_t *__restrict__ perm,
                                                              float *__restrict__ cost) {
    __shared__ int nv;
    const int64_t qb = blockIdx.x, i = qb * kBN + threadIdx.x;
    const int64_t o = i < m ? (perm ? (int64_t)perm[i] : i) : -1;  // (-1: padding)
    if (threadIdx.x == 0) nv = 0;
    __syncthreads();
    if (o >= 0) atomicAdd(&nv, 1);
    __syncthreads();
    if (o >= 0) cost[o] = bcost[qb] / (float)nv;
}

// ---- the sweep (persistent: one workgroup per CU)
// OT: outer (cross-tile) accumulator type.  Workgroup b walks the item range
// r(b) of the plan; consecutive ranges go to one XCD (blocks are dealt to the
// 8 XCDs round-robin), so an XCD's L2 sees neighbouring items.
template <class OT, int LOADERS = kPredictWaves / 2>
__global__ __launch_bounds__(kPredictThreads, 1) void predict_kernel(
    const float *__restrict__ aug, const float *__restrict__ kcoord, const int4 *__restrict__ desc,
    const unsigned short *__restrict__ tl, const int *__restrict__ seg, int P, int n_items, int nI,
    const float *__restrict__ qx, const float *__restrict__ qy, int64_t m, int64_t ldp, float cexp, float m0,
    float *__restrict__ part, float *__restrict__ mean) {
    __shared__ __attribute__((aligned(16))) float smem[kSmemFloats];
    const int bid = blockIdx.x;
    const int rng = (P % 8 == 0) ? (bid % 8) * (P / 8) + bid / 8 : bid;
    // (bounds are clamped so that a corrupt plan cannot address outside the buffers)
    const int k0 = max(seg[rng], 0), k1 = min(seg[rng + 1], n_items);
    if (k0 >= k1) return;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int g = lane >> 4;   // k within the step
    const int r = lane & 15;   // row within a 16-row block / query within the wave

    // LDS: two stages, then two descriptor windows and two tile-list windows
    // (1 KiB each), refilled one window ahead by LDS-DMA
    const int4 *dwin = reinterpret_cast<const int4 *>(smem + 2 * kStageFloats);
    const unsigned short *lwin = reinterpret_cast<const unsigned short *>(smem + 2 * kStageFloats + 512);

    // LDS-DMA (global_load_lds_dwordx4): each wave instruction moves 1 KiB,
    // lane-linear, no staging registers.  A stage = the 64 KiB [BK][BM] tile
    // (16 instructions per loader wave) + 768 B of per-k coordinates.  The
    // DMA is issued from inline asm so that hipcc does not see an LDS write
    // in flight: with a compiler-visible one pending it drains every ds_read
    // wait to lgkmcnt(0) (waiting on reads issued one instruction earlier)
    // instead of counting.  Every stage and window is retired by the
    // explicit vmcnt(0) + barrier at the end of each step.
    typedef __attribute__((address_space(3))) char lds_char;
    constexpr int kTileBytes = kTileFloats * 4, kStageBytes = kStageFloats * 4, kCBytes = 3 * kBK * 4;
    // Only the last LOADERS waves (one per SIMD) issue the stage, 16 pieces
    // each; the first four go straight from the barrier into their MFMAs
    // (1.8 % over every wave issuing 8, measured at C4).
    constexpr int kWaveStride = kTileBytes / LOADERS;  // bytes per loader wave per stage
    const int lw = wave - (kPredictWaves - LOADERS);    // loader index (< 0: not a loader)
    const bool loader = lw >= 0;
    const char *gA = reinterpret_cast<const char *>(aug) + (loader ? lw : 0) * 1024 + lane * 16;
    const char *gC = reinterpret_cast<const char *>(kcoord) + lane * 16;
    const char *gD = reinterpret_cast<const char *>(desc) + lane * 16;
    const char *gL = reinterpret_cast<const char *>(tl) + lane * 16;
    const uint32_t lds_smem = (uint32_t)(uintptr_t)(lds_char *)(smem);
    const uint32_t lds_wave = lds_smem + (uint32_t)__builtin_amdgcn_readfirstlane(loader ? lw : 0) * 1024u;
    const uint32_t lds_dwin = lds_smem + 2u * kStageBytes;
    const uint32_t lds_lwin = lds_dwin + 2048u;
#define SBO_DMA16(gsrc, ldst)                                                                           \
    do {                                                                                                \
        uint32_t keep_;                                                                                 \
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t" \
                     "s_mov_b32 m0, %0"                                                                 \
                     : "=&s"(keep_)                                                                     \
                     : "v"(gsrc), "s"(ldst)                                                             \
                     : "memory");                                                                       \
    } while (0)
#define SBO_STAGE(I_, t_, buf)                                                                          \
    do {                                                                                                \
        if (loader) {                                                                                   \
            const char *s_ = gA + (tile_start(I_) + (t_)) * (int64_t)kTileBytes;                       \
            const uint32_t d_ = lds_wave + (uint32_t)(buf) * kStageBytes;                               \
            _Pragma("unroll") for (int j = 0; j < kWaveStride / 1024; ++j)                              \
                SBO_DMA16(s_ + j * LOADERS * 1024, d_ + (uint32_t)(j * LOADERS * 1024));                \
        }                                                                                               \
        if (lw == 0 && lane < kCBytes / 16)                                                             \
            SBO_DMA16(gC + (int64_t)(t_) * kCBytes, lds_smem + (uint32_t)((buf) * kStageBytes + kTileBytes)); \
    } while (0)
    // descriptor window w (items [64w, 64w+64)) and tile-list window w
    // (entries [512w, 512w+512)), each into LDS buffer w & 1
#define SBO_DESC_WINDOW(w_)                                                                             \
    do {                                                                                                \
        if (lw == 1) SBO_DMA16(gD + (int64_t)(w_) * 1024, lds_dwin + (uint32_t)((w_) & 1) * 1024u);     \
    } while (0)
#define SBO_LIST_WINDOW(w_)                                                                             \
    do {                                                                                                \
        if (lw == 2) SBO_DMA16(gL + (int64_t)(w_) * 1024, lds_lwin + (uint32_t)((w_) & 1) * 1024u);     \
    } while (0)
    auto desc_at = [&](int k) {  // a descriptor from its (loaded) window; wave-uniform
        const int4 d = dwin[((k / kDescWindow) & 1) * kDescWindow + k % kDescWindow];
        const int I = min(max(__builtin_amdgcn_readfirstlane(d.x), 0), nI - 1);
        return make_int4(I, __builtin_amdgcn_readfirstlane(d.y), __builtin_amdgcn_readfirstlane(d.z),
                         __builtin_amdgcn_readfirstlane(d.w));
    };
    auto entry_off = [](const int4 &d) {
        return (uint64_t)(uint32_t)d.z | ((uint64_t)((uint32_t)d.w >> 16) << 32);
    };
    auto list_at = [&](uint64_t e, int I) {
        // (every level at full f32 precision here: the level code is ignored)
        const int t = __builtin_amdgcn_readfirstlane((int)lwin[((e / kListWindow) & 1) * kListWindow + e % kListWindow]) &
                      ((1 << kLevelShift) - 1);
        return min(t, kTilesPerRowBlockStep * (I + 1) - 1);
    };

    // ---- prologue: the first two windows of each kind, the first stage
    SBO_DESC_WINDOW(k0 / kDescWindow);
    SBO_DESC_WINDOW(k0 / kDescWindow + 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int4 dc = desc_at(k0);
    uint64_t e = entry_off(dc);
    SBO_LIST_WINDOW(e / kListWindow);
    SBO_LIST_WINDOW(e / kListWindow + 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    SBO_STAGE(dc.x, list_at(e, dc.x), 0);
    int64_t q = (int64_t)dc.y * kBN + wave * 16 + r;
    float xq = qx[q < m ? q : m - 1], yq = qy[q < m ? q : m - 1];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    OT outer[kRowBlocks][4];
#pragma unroll
    for (int rb = 0; rb < kRowBlocks; ++rb)
#pragma unroll
        for (int c = 0; c < 4; ++c) outer[rb][c] = (OT)0;
    double mu = 0.0;
    f32x4 acc[kRowBlocks];
    int k = k0, j = 0, cur = 0;
    for (;;) {
        const int cnt = dc.w & 0xffff;
        // the next step: (k, j+1), or the first tile of item k+1
        int kn = k, jn = j + 1;
        if (jn >= cnt) {
            kn = k + 1;
            jn = 0;
        }
        const bool more = kn < k1;
        int4 dn = dc;
        float xqn = xq, yqn = yq;
        if (more) {
            if (kn != k) {
                dn = desc_at(kn);
                if (kn % kDescWindow == 0) SBO_DESC_WINDOW(kn / kDescWindow + 1);
                const int64_t qn = (int64_t)dn.y * kBN + wave * 16 + r;
                xqn = qx[qn < m ? qn : m - 1];
                yqn = qy[qn < m ? qn : m - 1];
            }
            const uint64_t en = e + 1;
            if (en % kListWindow == 0) SBO_LIST_WINDOW(en / kListWindow + 1);
            SBO_STAGE(dn.x, list_at(en, dn.x), cur ^ 1);
        }
        // per-lane bases; every k step is a constant offset from them
        const float4 *pa = reinterpret_cast<const float4 *>(smem + cur * kStageFloats) + g * 16 + r;
        const float *pc = smem + cur * kStageFloats + kTileFloats + g * (kBK / 4);
        const int I = dc.x;
        if (I == nI - 1)
            tile_steps<true>(pa, pc, xq, yq, cexp, acc, mu);
        else
            tile_steps<false>(pa, pc, xq, yq, cexp, acc, mu);
#pragma unroll
        for (int rb = 0; rb < kRowBlocks; ++rb)
#pragma unroll
            for (int c = 0; c < 4; ++c) outer[rb][c] += (OT)acc[rb][c];
        if (j == cnt - 1) {
            // item done: column sums of V^2 over its rows; lanes l, l+16,
            // l+32, l+48 hold four row quarters of column l&15 of every block
            double s = 0.0;
#pragma unroll
            for (int rb = 0; rb < kRowBlocks; ++rb)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    s = fma((double)outer[rb][c], (double)outer[rb][c], s);
                    outer[rb][c] = (OT)0;
                }
            s += __shfl_xor(s, 16);
            s += __shfl_xor(s, 32);
            const bool writer = lane < 16 && q < m;
            if (writer) part[(int64_t)I * ldp + q] = (float)s;
            if (I == nI - 1) {
                mu += __shfl_xor(mu, 16);
                mu += __shfl_xor(mu, 32);
                if (writer) mean[q] = (float)((double)m0 + mu);
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
        j = jn;
        ++e;
        cur ^= 1;
    }
#undef SBO_STAGE
#undef SBO_DESC_WINDOW
#undef SBO_LIST_WINDOW
#undef SBO_DMA16
}

// ------------------------------------------------------ a6+a7+a10 acquire
__device__ __forceinline__ bool key_better(double as, int64_t ai, double bs, int64_t bi) {
    if (ai < 0) return false;
    if (bi < 0) return true;
    if (as > bs) return true;
    if (as < bs) return false;
    return ai < bi;
}

__device__ __forceinline__ void block_reduce_key(double &s, int64_t &i, sbo_key *out) {
    __shared__ double ss[kAcqThreads / 64];
    __shared__ int64_t si[kAcqThreads / 64];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const double os = __shfl_xor(s, off);
        const int64_t oi = __shfl_xor(i, off);
        if (key_better(os, oi, s, i)) { s = os; i = oi; }
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { ss[w] = s; si[w] = i; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < (int)(blockDim.x >> 6); ++k)
            if (key_better(ss[k], si[k], s, i)) { s = ss[k]; i = si[k]; }
        out->score = s;
        out->idx = i;
    }
}

// node.cpp:411-416 and :409 in IEEE double, no contraction:
//   confidence = beta * std;  lo = mu - confidence;  hi = mu + confidence;  S = lo > f_min
// T = float (the tick's own f32 outputs, widened exactly) or double (the
// node's f64 mu_/std_, node.cpp:129-130, :641-643)
template <typename T>
__device__ __forceinline__ void compute_sets_one(T mu, T sd, double beta, double f_min,
                                                 double &lo, double &hi, bool &safe) {
    const double c = __dmul_rn(beta, (double)sd);
    lo = __dsub_rn((double)mu, c);
    hi = __dadd_rn((double)mu, c);
    safe = lo > f_min;
}

template <class PT>
__global__ __launch_bounds__(kAcqThreads) void acquire_kernel(
    const PT *__restrict__ part, const PT *__restrict__ mean, int nI, int64_t ldp, int64_t m,
    double sf2, double beta, double f_min, int score_kind, int64_t index_offset,
    const int32_t *__restrict__ perm, float *__restrict__ mu_out, float *__restrict__ sd_out,
    double *__restrict__ lo_out, double *__restrict__ hi_out, uint8_t *__restrict__ safe_out,
    sbo_key *__restrict__ keys) {
    const int64_t i = (int64_t)blockIdx.x * kAcqThreads + threadIdx.x;
    double bs = 0.0;
    int64_t bi = -1;
    // (perm -1: a padded grid-patch position, no output)
    if (i < m && (!perm || perm[i] >= 0)) {
        // the row blocks' partials, summed in f64 in ascending I; read eight
        // at a time so their loads are in flight together (same sum order)
        double s = 0.0;
        int I = 0;
        for (; I + 8 <= nI; I += 8) {
            PT v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)(I + u) * ldp + i];
#pragma unroll
            for (int u = 0; u < 8; ++u) s += (double)v[u];
        }
        for (; I < nI; ++I) s += (double)part[(int64_t)I * ldp + i];
        double vd = sf2 - s;
        float var = vd > 0.0 ? (float)vd : 0.0f;
        const float sd = __fsqrt_rn(var);
        const float mu = (float)mean[i];
        const int64_t o = perm ? (int64_t)perm[i] : i;  // caller's index of sweep position i
        if (mu_out) mu_out[o] = mu;
        if (sd_out) sd_out[o] = sd;
        double lo, hi;
        bool safe;
        compute_sets_one(mu, sd, beta, f_min, lo, hi, safe);
        if (lo_out) lo_out[o] = lo;
        if (hi_out) hi_out[o] = hi;
        if (safe_out) safe_out[o] = safe ? 1 : 0;
        const double score = score_kind == SBO_SCORE_UCB ? hi : __dsub_rn(hi, lo);
        if (safe && score == score) { bs = score; bi = index_offset + o; }
    }
    block_reduce_key(bs, bi, keys + blockIdx.x);
}

template <typename T>
__global__ __launch_bounds__(kAcqThreads) void sets_kernel(const T *__restrict__ mu,
                                                           const T *__restrict__ sd, int64_t m,
                                                           double beta, double f_min,
                                                           double *__restrict__ lo,
                                                           double *__restrict__ hi,
                                                           uint8_t *__restrict__ safe) {
    const int64_t i = (int64_t)blockIdx.x * kAcqThreads + threadIdx.x;
    if (i >= m) return;
    double l, h;
    bool s;
    compute_sets_one(mu[i], sd[i], beta, f_min, l, h, s);
    if (lo) lo[i] = l;
    if (hi) hi[i] = h;
    if (safe) safe[i] = s ? 1 : 0;
}

__global__ __launch_bounds__(kAcqThreads) void argmax_kernel(const double *__restrict__ score,
                                                             const uint8_t *__restrict__ mask,
                                                             int64_t m, int64_t index_offset,
                                                             sbo_key *__restrict__ keys) {
    const int64_t i = (int64_t)blockIdx.x * kAcqThreads + threadIdx.x;
    double bs = 0.0;
    int64_t bi = -1;
    if (i < m && (!mask || mask[i])) {
        const double v = score[i];
        if (v == v) { bs = v; bi = index_offset + i; }
    }
    block_reduce_key(bs, bi, keys + blockIdx.x);
}

__global__ __launch_bounds__(kAcqThreads) void reduce_keys_kernel(const sbo_key *__restrict__ keys,
                                                                  int64_t nb,
                                                                  sbo_key *__restrict__ out) {
    double bs = 0.0;
    int64_t bi = -1;
    for (int64_t k = threadIdx.x; k < nb; k += kAcqThreads) {
        const sbo_key v = keys[k];
        if (key_better(v.score, v.idx, bs, bi)) { bs = v.score; bi = v.idx; }
    }
    block_reduce_key(bs, bi, out);
}

}  // namespace

// ---------------------------------------------------------------- launchers
hipError_t launch_rbf_fill(hipStream_t s, const float *xa, const float *ya, int64_t ma, const float *xb,
                           const float *yb, int64_t mb, int64_t ld, float ell, float sf2, float sn2, bool diag,
                           float *K) {
    const float c = -1.0f / (2.0f * ell * ell);
    const dim3 grid((unsigned)((ma + 1023) / 1024), (unsigned)((mb + kFillCols - 1) / kFillCols));
    const bool vec = (ld % 4 == 0) && ((reinterpret_cast<uintptr_t>(K) & 15) == 0) &&
                     ((reinterpret_cast<uintptr_t>(xa) & 15) == 0) &&
                     ((reinterpret_cast<uintptr_t>(ya) & 15) == 0);
    if (vec)
        hipLaunchKernelGGL(rbf_fill_kernel<true>, grid, dim3(256), 0, s, xa, ya, ma, xb, yb, mb, ld, c, sf2, sn2,
                           (int)diag, K);
    else
        hipLaunchKernelGGL(rbf_fill_kernel<false>, grid, dim3(256), 0, s, xa, ya, ma, xb, yb, mb, ld, c, sf2, sn2,
                           (int)diag, K);
    return hipGetLastError();
}

hipError_t launch_sub_scalar(hipStream_t s, const float *in, float v, int64_t n, float *out) {
    hipLaunchKernelGGL(sub_scalar_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in, v, n, out);
    return hipGetLastError();
}

hipError_t launch_copy_lower(hipStream_t s, const float *src, int64_t ld_src, int64_t n, float *dst,
                             int64_t ld_dst) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(copy_lower_kernel, dim3((unsigned)((n + 255) / 256), (unsigned)std::min<int64_t>(n, kMaxGridY)),
                       dim3(256), 0, s, src, ld_src, n, dst, ld_dst);
    return hipGetLastError();
}

hipError_t launch_pack_tiles(hipStream_t s, const double *Linv, int64_t ld, int64_t n, int64_t npad, int64_t I0,
                             double sf2, float *aug) {
    const int64_t nI = npad / kBM;
    if (I0 >= nI) return hipSuccess;
    hipLaunchKernelGGL(pack_operand_kernel<double>, dim3((unsigned)(nI * kTilesPerRowBlockStep), (unsigned)(nI - I0)),
                       dim3(256), 0, s, Linv, ld, n, sf2, I0, aug);
    return hipGetLastError();
}

hipError_t launch_pack_kcoord(hipStream_t s, const float *x, const float *y, const float *alpha, int64_t n,
                              int64_t npad, double sf2, float *kcoord) {
    hipLaunchKernelGGL(pack_kcoord_kernel, dim3((unsigned)((npad + 255) / 256)), dim3(256), 0, s, x, y, alpha, n, npad,
                       (float)sf2, kcoord);
    return hipGetLastError();
}

template <class T>
hipError_t launch_pack_operand_t(hipStream_t s, const T *Linv, int64_t ld, int64_t n, int64_t npad, int64_t I0,
                                 double sf2, const float *x, const float *y, const float *alpha, float *aug,
                                 float *kcoord) {
    const int64_t nI = npad / kBM;
    if (I0 < nI) {
        hipLaunchKernelGGL(pack_operand_kernel<T>, dim3((unsigned)(nI * kTilesPerRowBlockStep), (unsigned)(nI - I0)),
                           dim3(256), 0, s, Linv, ld, n, (T)sf2, I0, aug);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(pack_kcoord_kernel, dim3((unsigned)((npad + 255) / 256)), dim3(256), 0, s, x, y,
                       alpha, n, npad, (float)sf2, kcoord);
    return hipGetLastError();
}

hipError_t launch_pack_operand(hipStream_t s, const float *Linv, int64_t ld, int64_t n, int64_t npad, int64_t I0,
                               double sf2, const float *x, const float *y, const float *alpha, float *aug,
                               float *kcoord) {
    return launch_pack_operand_t<float>(s, Linv, ld, n, npad, I0, sf2, x, y, alpha, aug, kcoord);
}

hipError_t launch_pack_operand(hipStream_t s, const double *Linv, int64_t ld, int64_t n, int64_t npad, int64_t I0,
                               double sf2, const float *x, const float *y, const float *alpha, float *aug,
                               float *kcoord) {
    return launch_pack_operand_t<double>(s, Linv, ld, n, npad, I0, sf2, x, y, alpha, aug, kcoord);
}

hipError_t launch_widen(hipStream_t s, const float *src, int64_t ld_src, int64_t m, int64_t n, bool lower,
                        double *dst, int64_t ld_dst) {
    if (m <= 0 || n <= 0) return hipSuccess;
    hipLaunchKernelGGL(widen_kernel, dim3((unsigned)((m + 255) / 256), (unsigned)std::min<int64_t>(n, kMaxGridY)),
                       dim3(256), 0, s, src, ld_src, m, n, lower ? 1 : 0, dst, ld_dst);
    return hipGetLastError();
}

hipError_t launch_row_l1(hipStream_t s, const float *aug, int64_t npad, int64_t I0, double *row_l1) {
    const int64_t nI = npad / kBM;
    if (I0 >= nI) return hipSuccess;
    hipError_t e = hipMemsetAsync(row_l1 + I0 * kBM, 0, sizeof(double) * (size_t)((nI - I0) * kBM), s);
    if (e != hipSuccess) return e;
    const int64_t chunks = (nI * kTilesPerRowBlockStep + kRowL1Tiles - 1) / kRowL1Tiles;
    hipLaunchKernelGGL(row_l1_kernel, dim3((unsigned)chunks, (unsigned)(nI - I0)), dim3(kBM), 0, s, aug, I0, row_l1);
    return hipGetLastError();
}

hipError_t launch_chol_diag(hipStream_t s, float *A, int64_t ld, int kb, int64_t k0, int *info, int version) {
    if (kb <= 0 || kb > kCholNB) return hipErrorInvalidValue;
    if (version == 1)
        hipLaunchKernelGGL(chol_diag_ll_kernel, dim3(1), dim3(256), 0, s, A, ld, kb, k0, info);
    else if (version == 2)
        hipLaunchKernelGGL(chol_diag_mfma_kernel, dim3(1), dim3(256), 0, s, A, ld, kb, k0, info);
    else
        hipLaunchKernelGGL(chol_diag_kernel, dim3(1), dim3(256), 0, s, A, ld, kb, k0, info);
    return hipGetLastError();
}

hipError_t launch_chol_update(hipStream_t s, const float *P, const float *Q, int64_t ld, int64_t m, int64_t nc,
                              int64_t K, bool lower, float *C) {
    if (m < 0 || nc < 0 || K < 0 || m > INT32_MAX / 2 || nc > INT32_MAX / 2 || K > INT32_MAX / 2 || (lower && nc != m) ||
        K % kUpBK != 0)
        return hipErrorInvalidValue;
    if (m == 0 || nc == 0 || K == 0) return hipSuccess;
    const int64_t nti = (m + kUpBM - 1) / kUpBM, ntj = (nc + kUpBM - 1) / kUpBM;
    const int64_t tiles = lower ? nti * (nti + 1) / 2 : nti * ntj;
    if (tiles > INT32_MAX) return hipErrorInvalidValue;
    hipLaunchKernelGGL(chol_update_kernel, dim3((unsigned)tiles), dim3(256), 0, s, P, Q, ld, (int)m, (int)nc, (int)K,
                       lower ? 1 : 0, C);
    return hipGetLastError();
}

hipError_t launch_chol_trsm(hipStream_t s, const float *L11, int64_t ld, int kb, float *A21, int64_t m2, int version) {
    if (kb <= 0 || kb > kCholNB || m2 < 0) return hipErrorInvalidValue;
    if (m2 == 0) return hipSuccess;
    if (version == 1)
        hipLaunchKernelGGL(chol_trsm_ll_kernel, dim3((unsigned)((m2 + kCholNB - 1) / kCholNB)), dim3(2 * kCholNB), 0,
                           s, L11, ld, kb, A21, m2);
    else if (version == 2)
        hipLaunchKernelGGL(chol_trsm_mfma_kernel, dim3((unsigned)((m2 + kCholNB - 1) / kCholNB)), dim3(2 * kCholNB), 0,
                           s, L11, ld, kb, A21, m2);
    else
        hipLaunchKernelGGL(chol_trsm_kernel, dim3((unsigned)((m2 + kCholNB - 1) / kCholNB)), dim3(2 * kCholNB), 0, s,
                           L11, ld, kb, A21, m2);
    return hipGetLastError();
}

hipError_t launch_pack_tile_norms(hipStream_t s, const double *Linv, int64_t ld, int64_t n, int64_t npad, int64_t I0,
                                  double sf2, float *aug, float4 *lgn) {
    const int64_t nI = npad / kBM;
    const int64_t t0 = tile_start(I0), t1 = tile_start(nI);
    if (t1 <= t0) return hipSuccess;
    hipLaunchKernelGGL(tile_norm_kernel<true>, dim3((unsigned)(t1 - t0)), dim3(kBM), 0, s, aug, t0, lgn, Linv, ld, n,
                       sf2, aug);
    return hipGetLastError();
}

hipError_t launch_tile_norms(hipStream_t s, const float *aug, int64_t npad, int64_t I0, float4 *lgn) {
    const int64_t nI = npad / kBM;
    const int64_t t0 = tile_start(I0), t1 = tile_start(nI);
    if (t1 <= t0) return hipSuccess;
    hipLaunchKernelGGL(tile_norm_kernel<false>, dim3((unsigned)(t1 - t0)), dim3(kBM), 0, s, aug, t0, lgn, nullptr,
                       (int64_t)0, (int64_t)0, 0.0, nullptr);
    return hipGetLastError();
}

hipError_t launch_widen_sub(hipStream_t s, const float *in, double v, int64_t n, double *d) {
    hipLaunchKernelGGL(widen_sub_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in, v, n, d);
    return hipGetLastError();
}

hipError_t launch_narrow(hipStream_t s, const double *d, int64_t n, float *out) {
    hipLaunchKernelGGL(narrow_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d, n, out);
    return hipGetLastError();
}

size_t alpha_work_bytes(int64_t n) { return sizeof(double) * (size_t)((n + kAlK - 1) / kAlK) * (size_t)n; }

hipError_t launch_alpha_f64(hipStream_t s, const double *X, int64_t ld, int64_t n, const float *obs, double m0,
                            double *z, double *alpha, double *work) {
    if (n <= 0) return hipSuccess;
    const dim3 g1((unsigned)((n + kAlRows - 1) / kAlRows), (unsigned)((n + kAlK - 1) / kAlK));
    hipLaunchKernelGGL(alpha_z_kernel, g1, dim3(256), 0, s, X, ld, n, obs, m0, work);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(alpha_z_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, work, n, z);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(alpha_xtz_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, X, ld, n, z, alpha);
    return hipGetLastError();
}

hipError_t launch_row_dot(hipStream_t s, const double *A, int64_t ld, int64_t rows, int64_t n, const double *x,
                          double *out) {
    if (rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(row_dot_kernel, dim3((unsigned)rows), dim3(256), 0, s, A, ld, n, x, out);
    return hipGetLastError();
}

hipError_t launch_narrow_2d(hipStream_t s, const double *d, int64_t ldd, int64_t m, int64_t n, float *out,
                            int64_t ldo) {
    if (m <= 0 || n <= 0) return hipSuccess;
    hipLaunchKernelGGL(narrow_2d_kernel, dim3((unsigned)((m + 255) / 256), (unsigned)std::min<int64_t>(n, kMaxGridY)),
                       dim3(256), 0, s, d, ldd, m, n, out, ldo);
    return hipGetLastError();
}

hipError_t launch_narrow_strided(hipStream_t s, const double *d, int64_t n, float *out, int64_t stride) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(narrow_strided_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d, n, out, stride);
    return hipGetLastError();
}

hipError_t launch_tile_boxes(hipStream_t s, const float *x, const float *y, int64_t n, int64_t npad, float4 *kbox) {
    const int64_t nt = npad / kBK;
    hipLaunchKernelGGL(tile_box_kernel, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, s, x, y, n, nt, kbox);
    return hipGetLastError();
}

namespace {
struct PlanLayout {
    size_t key, scan, thr, desc, tl, seg, temp, temp_bytes, wkey, wscan, lvcnt, rec, bits;
    // XCD-interleaved order (P % 8 == 0): the sweep reads desc2 / tl2 / seg2
    bool xcd;
    size_t xseg, pos_of, cnt2, off2, desc2, tl2, seg2, temp2, temp2_bytes;
    size_t total;
};

bool xcd_interleave(int P) { return P >= 8 && P % 8 == 0; }

PlanLayout plan_layout(int64_t nI, int64_t nQ, int P) {
    const int64_t items = nI * nQ;
    const int64_t cap = 2 * nI * (nI + 1) * nQ;  // every tile of every item (the dense sweep)
    PlanLayout L{};
    size_t o = 0;
    auto take = [&](size_t b) {
        const size_t at = o;
        o = (o + b + 255) / 256 * 256;
        return at;
    };
    L.key = take(8 * (size_t)items);
    L.scan = take(8 * (size_t)items);
    L.thr = take((size_t)items);
    L.wkey = take(8 * (size_t)items);
    L.wscan = take(8 * (size_t)items);
    L.lvcnt = take(8 * 3 * 4 * (size_t)kPlanWriteBlocks);
    L.bits = take(8 * 3 * (size_t)items * (size_t)plan_chunks((int)nI));
    L.desc = take(16 * (size_t)(items + 2 * kDescWindow));
    L.tl = take(2 * (size_t)(cap + 2 * kListWindow));
    L.seg = take(4 * (size_t)(P + 1));
    L.rec = take(16 * (size_t)(cap + 2 * kRecWindow));
    size_t tb = 0;
    (void)rocprim::inclusive_scan(nullptr, tb, (const unsigned long long *)nullptr, (unsigned long long *)nullptr,
                                  (size_t)items, rocprim::plus<unsigned long long>());
    L.temp = take(tb);
    L.temp_bytes = tb;
    L.xcd = xcd_interleave(P);
    if (L.xcd) {
        L.xseg = take(4 * 9);
        L.pos_of = take(4 * (size_t)items);
        L.cnt2 = take(8 * (size_t)items);
        L.off2 = take(8 * (size_t)items);
        L.desc2 = take(16 * (size_t)(items + 2 * kDescWindow));
        L.tl2 = take(2 * (size_t)(cap + 2 * kListWindow));
        L.seg2 = take(4 * (size_t)(P + 1));
        size_t t2 = 0;
        (void)rocprim::exclusive_scan(nullptr, t2, (const unsigned long long *)nullptr, (unsigned long long *)nullptr,
                                      0ull, (size_t)items, rocprim::plus<unsigned long long>());
        L.temp2 = take(t2);
        L.temp2_bytes = t2;
    }
    L.total = o;
    return L;
}

// k-tiles farther than this squared distance give c*d^2 < -L, i.e. every K*
// entry < 2^-L (0.1% margin over the kernel's rounding); L >= 150 means every
// such entry is exactly +0.0 in f32
float cutoff_d2(int L, double ce) { return L > 0 ? (float)((double)L / -ce * 1.001) : -1.0f; }
double exp2_coef(float ell) { return -1.0 / (2.0 * (double)ell * (double)ell * 0.69314718055994530942); }
}  // namespace

size_t predict_work_bytes(int64_t npad, int64_t m, int P) {
    return plan_layout(npad / kBM, (m + kBN - 1) / kBN, P).total;
}

hipError_t launch_plan(hipStream_t s, const float4 *kbox, int64_t npad, const float *qx, const float *qy, int64_t m,
                       int64_t ldp, float ell, float m0, const SkipPlan &skip, float *part, float *mean,
                       unsigned long long *tiles_done, int P, void *work, size_t work_bytes) {
    const int nI = (int)(npad / kBM);
    const int64_t nQ = (m + kBN - 1) / kBN;
    const int64_t items = (int64_t)nI * nQ;
    if (m <= 0 || nI <= 0) return hipSuccess;
    // key fields: items < 2^24, every kept-tile count < 2^40; tile index < 2^14 (level code above)
    if (nQ > 0x7fffffff || items >= (1ll << (64 - kPlanKeyShift)) ||
        2 * (int64_t)nI * (nI + 1) * nQ >= (1ll << kPlanKeyShift) || kTilesPerRowBlockStep * (int64_t)nI > (1 << kLevelShift) - 1)
        return hipErrorInvalidValue;
    const PlanLayout L = plan_layout(nI, nQ, P);
    if (work_bytes < L.total) return hipErrorInvalidValue;
    if (skip.order_blk != 0 && ((skip.order_blk >> 8) < 1 || (skip.order_blk & 255) < 1 || (skip.order_blk >> 16) != 0))
        return hipErrorInvalidValue;
    char *w = static_cast<char *>(work);
    auto *key = reinterpret_cast<unsigned long long *>(w + L.key);
    auto *scan = reinterpret_cast<unsigned long long *>(w + L.scan);
    auto *thr = reinterpret_cast<unsigned char *>(w + L.thr);
    auto *desc = reinterpret_cast<int4 *>(w + L.desc);
    auto *tl = reinterpret_cast<unsigned short *>(w + L.tl);
    auto *seg = reinterpret_cast<int *>(w + L.seg);
    auto *wkey = reinterpret_cast<unsigned long long *>(w + L.wkey);
    auto *wscan = reinterpret_cast<unsigned long long *>(w + L.wscan);
#ifdef SBO_DIAG
    if (const char *ev = getenv("SBO_MEAN_W")) {
        unsigned v[3] = {kMeanWeight0, kMeanWeight1, kMeanWeight2};
        if (sscanf(ev, "%u,%u,%u", &v[0], &v[1], &v[2]) == 3)
            (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_mean_w), v, sizeof(v), 0, hipMemcpyHostToDevice, s);
    }
    if (const char *ev = getenv("SBO_RB_SLOPE")) {
        const unsigned v = (unsigned)std::max(0, atoi(ev));
        (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_rb_slope), &v, sizeof(v), 0, hipMemcpyHostToDevice, s);
    }
#endif
    const double ce = exp2_coef(ell);
    const float cexp = (float)ce;
    const float skip_d2 = cutoff_d2(skip.L, ce);
    const float skip_d2_mean = skip.L > 0 && skip.L_mean > skip.L ? cutoff_d2(skip.L_mean, ce) : skip_d2;
    const float4 *lgn = skip.L > 0 ? skip.lgn : nullptr;
    const int levels = lgn ? skip.levels : 0;
    auto *bits = reinterpret_cast<unsigned long long *>(w + L.bits);
    const int nc = std::min(kTilesPerRowBlockStep * nI, kPlanD2);
    const size_t plan_lds = 4 * (size_t)kPlanWaves * kPlanBinCache + 8 * (size_t)nc;
    hipLaunchKernelGGL(plan_count_kernel, dim3((unsigned)nQ), dim3(kPlanThreads), plan_lds, s, kbox, skip.kcoord, lgn,
                       levels, make_float2(skip.lvl_key[0], skip.lvl_key[1]), nI,
                       nQ, qx, qy,
                       m, cexp, skip_d2, skip_d2_mean, skip.lg_tau_v, m0, ldp, part, mean, key, thr, wkey, bits,
                       skip.wide ? 1 : 0, skip.order_blk);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    size_t tb = L.temp_bytes;
    e = rocprim::inclusive_scan(w + L.temp, tb, key, scan, (size_t)items, rocprim::plus<unsigned long long>(), s);
    if (e != hipSuccess) return e;
    tb = L.temp_bytes;
    e = rocprim::inclusive_scan(w + L.temp, tb, wkey, wscan, (size_t)items, rocprim::plus<unsigned long long>(), s);
    if (e != hipSuccess) return e;
    const int64_t wblocks = std::min<int64_t>((items + 3) / 4, kPlanWriteBlocks);
    hipLaunchKernelGGL(plan_write_kernel, dim3((unsigned)wblocks), dim3(256), 0, s, nI, nQ, key, scan, bits,
                       desc, tl, skip.prod_full, tiles_done ? reinterpret_cast<unsigned long long *>(w + L.lvcnt) : nullptr,
                       skip.order_blk);
    if (tiles_done)
        hipLaunchKernelGGL(plan_counts_reduce_kernel, dim3(1), dim3(256), 0, s,
                           reinterpret_cast<const unsigned long long *>(w + L.lvcnt), wblocks * 4, tiles_done + 1);
    auto *rec = reinterpret_cast<int4 *>(w + L.rec);
    if (!L.xcd) {
        hipLaunchKernelGGL(plan_seg_kernel, dim3(1), dim3(256), 0, s, scan, items, desc, P, seg, tiles_done, wkey,
                           wscan, nI, nQ, skip.order_blk);
        if (skip.records)
            hipLaunchKernelGGL(plan_rec_kernel, dim3((unsigned)((items + 3) / 4)), dim3(256), 0, s, scan, items, desc,
                               tl, rec);
        return hipGetLastError();
    }
    auto *xseg = reinterpret_cast<int *>(w + L.xseg);
    auto *pos_of = reinterpret_cast<int *>(w + L.pos_of);
    auto *cnt2 = reinterpret_cast<unsigned long long *>(w + L.cnt2);
    auto *off2 = reinterpret_cast<unsigned long long *>(w + L.off2);
    auto *desc2 = reinterpret_cast<int4 *>(w + L.desc2);
    auto *tl2 = reinterpret_cast<unsigned short *>(w + L.tl2);
    auto *seg2 = reinterpret_cast<int *>(w + L.seg2);
    const int G = P / 8;
    // (positions past the last non-empty item keep count 0 for the scan)
    e = hipMemsetAsync(cnt2, 0, 8 * (size_t)items, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(plan_seg_kernel, dim3(1), dim3(256), 0, s, scan, items, desc, 8, xseg, tiles_done, wkey, wscan,
                       nI, nQ, skip.order_blk);
    hipLaunchKernelGGL(plan_perm_kernel, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, s, scan, items, desc,
                       xseg, G, pos_of, cnt2);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    size_t t2 = L.temp2_bytes;
    e = rocprim::exclusive_scan(w + L.temp2, t2, cnt2, off2, 0ull, (size_t)items,
                                rocprim::plus<unsigned long long>(), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(plan_move_kernel, dim3((unsigned)((items + 3) / 4)), dim3(256), 0, s, scan, items, desc, tl,
                       pos_of, off2, desc2, tl2, skip.records ? rec : nullptr);
    hipLaunchKernelGGL(plan_seg2_kernel, dim3(1), dim3(256), 0, s, xseg, G, P, seg2);
    return hipGetLastError();
}

void plan_views(int64_t npad, int64_t m, int P, const void *work, const int4 **desc, const unsigned short **tl,
                const int **seg, const int4 **rec) {
    const PlanLayout L = plan_layout(npad / kBM, (m + kBN - 1) / kBN, P);
    const char *w = static_cast<const char *>(work);
    *desc = reinterpret_cast<const int4 *>(w + (L.xcd ? L.desc2 : L.desc));
    *tl = reinterpret_cast<const unsigned short *>(w + (L.xcd ? L.tl2 : L.tl));
    *seg = reinterpret_cast<const int *>(w + (L.xcd ? L.seg2 : L.seg));
    if (rec) *rec = reinterpret_cast<const int4 *>(w + L.rec);
}

float exp2_coef_f(float ell) { return (float)exp2_coef(ell); }

hipError_t launch_plan_cost(hipStream_t s, int64_t npad, int64_t m, int P, const void *work, const int32_t *perm,
                            float *bcost, float *cost) {
    const int nI = (int)(npad / kBM);
    const int64_t nQ = (m + kBN - 1) / kBN;
    if (m <= 0 || nI <= 0) return hipSuccess;
    const PlanLayout L = plan_layout(nI, nQ, P);
    const auto *wkey = reinterpret_cast<const unsigned long long *>(static_cast<const char *>(work) + L.wkey);
    hipLaunchKernelGGL(plan_block_cost_kernel, dim3((unsigned)((nQ + 255) / 256)), dim3(256), 0, s, wkey, nI, nQ,
                       bcost);
    hipLaunchKernelGGL(plan_query_cost_kernel, dim3((unsigned)nQ), dim3(kBN), 0, s, bcost, m, perm, cost);
    return hipGetLastError();
}

hipError_t launch_predict(hipStream_t s, const float *aug, const float *kcoord, int64_t npad, const float *qx,
                          const float *qy, int64_t m, int64_t ldp, float ell, float m0, float *part, float *mean,
                          int variant, int P, const void *work) {
    const int nI = (int)(npad / kBM);
    const int64_t nQ = (m + kBN - 1) / kBN;
    if (m <= 0 || nI <= 0) return hipSuccess;
    const int4 *desc = nullptr;
    const unsigned short *tl = nullptr;
    const int *seg = nullptr;
    plan_views(npad, m, P, work, &desc, &tl, &seg);
    const float cexp = (float)exp2_coef(ell);
#define SBO_PREDICT_ARGS aug, kcoord, desc, tl, seg, P, (int)(nI * nQ), nI, qx, qy, m, ldp, cexp, m0, part, mean
    switch (variant) {
        case 1: hipLaunchKernelGGL((predict_kernel<double>), dim3((unsigned)P), dim3(kPredictThreads), 0, s, SBO_PREDICT_ARGS); break;
        default: hipLaunchKernelGGL((predict_kernel<float>), dim3((unsigned)P), dim3(kPredictThreads), 0, s, SBO_PREDICT_ARGS); break;
    }
#undef SBO_PREDICT_ARGS
    return hipGetLastError();
}

hipError_t launch_acquire(hipStream_t s, const float *part, const float *mean, int nI, int64_t ldp,
                          int64_t m, float sf2, double beta, double f_min, int score_kind,
                          int64_t index_offset, const int32_t *perm, float *mu, float *sd, double *lo,
                          double *hi, uint8_t *safe, sbo_key *block_keys) {
    hipLaunchKernelGGL(acquire_kernel<float>, dim3((unsigned)acq_blocks(m)), dim3(kAcqThreads), 0, s, part, mean,
                       nI, ldp, m, (double)sf2, beta, f_min, score_kind, index_offset, perm, mu, sd, lo, hi, safe,
                       block_keys);
    return hipGetLastError();
}

hipError_t launch_acquire(hipStream_t s, const double *part, const double *mean, int nI, int64_t ldp,
                          int64_t m, double sf2, double beta, double f_min, int score_kind,
                          int64_t index_offset, const int32_t *perm, float *mu, float *sd, double *lo,
                          double *hi, uint8_t *safe, sbo_key *block_keys) {
    hipLaunchKernelGGL(acquire_kernel<double>, dim3((unsigned)acq_blocks(m)), dim3(kAcqThreads), 0, s, part, mean,
                       nI, ldp, m, sf2, beta, f_min, score_kind, index_offset, perm, mu, sd, lo, hi, safe,
                       block_keys);
    return hipGetLastError();
}

hipError_t launch_sets(hipStream_t s, const float *mu, const float *sd, int64_t m, double beta,
                       double f_min, double *lo, double *hi, uint8_t *safe) {
    hipLaunchKernelGGL(sets_kernel<float>, dim3((unsigned)acq_blocks(m)), dim3(kAcqThreads), 0, s, mu, sd, m, beta,
                       f_min, lo, hi, safe);
    return hipGetLastError();
}

hipError_t launch_sets(hipStream_t s, const double *mu, const double *sd, int64_t m, double beta,
                       double f_min, double *lo, double *hi, uint8_t *safe) {
    hipLaunchKernelGGL(sets_kernel<double>, dim3((unsigned)acq_blocks(m)), dim3(kAcqThreads), 0, s, mu, sd, m,
                       beta, f_min, lo, hi, safe);
    return hipGetLastError();
}

hipError_t launch_argmax_blocks(hipStream_t s, const double *score, const uint8_t *mask, int64_t m,
                                int64_t index_offset, sbo_key *block_keys) {
    hipLaunchKernelGGL(argmax_kernel, dim3((unsigned)acq_blocks(m)), dim3(kAcqThreads), 0, s, score, mask,
                       m, index_offset, block_keys);
    return hipGetLastError();
}

hipError_t launch_reduce_keys(hipStream_t s, const sbo_key *keys, int64_t nblocks, sbo_key *out) {
    hipLaunchKernelGGL(reduce_keys_kernel, dim3(1), dim3(kAcqThreads), 0, s, keys, nblocks, out);
    return hipGetLastError();
}

}  // namespace sbo
