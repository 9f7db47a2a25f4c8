// ozgemm.hip -- an f64 GEMM emulated on the int8 matrix cores (Ozaki-style
// slices), for the fit's f64 triangular inverse (SBO_OPT_INV_OZ, round 4).
//
// Why: the inverse's products are rocBLAS dgemms at 0.93 of the 78.6 TF f64
// MFMA peak (~24 ms of the C4 fit, ~20 at the peak);
// v_mfma_i32_16x16x64_i8 runs 2x the bf16 rate (5 POPS) and sums exactly.
// C = alpha op(A) B, A (m x K) and B (K x n) column-major f64:
//   each row of A and each column of B gets a power of two 2^e > 1.01 max|.|
//   over its K entries and the integer X = rint(a 2^(8 ND - 1 - e)) (|X| <
//   2^(8 ND - 1) / 1.01) cut into ND balanced base-256 digits (the bytes of X +
//   0x80..80, less 128 but for the top one: every digit in [-128, 127]);
//   level L = s + u < ND of the digit products (s of A, u of B) is summed
//   EXACTLY in int32 over all K (at most ND pairs of 64 products of <= 2^14
//   per MFMA, K <= 16384: < 2^31), the levels combined once per element in
//   f64 at the end: C = alpha 2^(eA + eB - 8 ND - 6) sum_L l_L 256^(ND-1-L).
// The dropped levels (s + u >= ND) and the rounding of X bound the error by
// about ND K 2^(14 - 8 ND - 2) of K max|row| max|col| -- relative to the
// row and column maxima, not to |A| |B| elementwise as a dgemm's is.
//
// Operand layout (gz_max_kernel, gz_digits_kernel): rows of 16 (A's rows, B's columns) by
// k-blocks of 64, [row block][k block][digit][1 KiB] with lane r + 16 g of a
// 1 KiB piece holding row r's bytes k = 16 g .. 16 g + 15 -- the MFMA's
// fragment order, so a stage is copied linearly by LDS-DMA and every operand
// read is one conflict-free ds_read_b128.
// GEMM (gz_gemm_kernel): workgroup = 128 rows of A x 64 columns of B, four
// waves of 32 x 64 (two A blocks held in registers, the four B blocks loaded
// in turn), ND x 8 int32 accumulator blocks per wave; a stage is one k-block
// (12 ND KiB), double buffered, one barrier per k-block.  Lower-triangular
// operands start / stop the k loop at the tile's diagonal.
#include <cstdint>
#include <type_traits>

#include "sbo_internal.hpp"

namespace sbo {
namespace {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
constexpr unsigned kGzVec4 = 1u << 30;   // (internal) the f32 epilogue may use 16-B accesses

constexpr int kGzTM = 128;   // rows of A per workgroup
constexpr int kGzTN = 64;    // columns of B per workgroup
constexpr int kGzNPad = 128; // B's columns padded to (the 128-column tiles of gz_run at <= 5 digits)
constexpr int kGzBK = 64;    // k per stage
constexpr int kGzMaxK = 16384;

__device__ __forceinline__ i32x4 mfma_i8(i32x4 a, i32x4 b, i32x4 c) {
    return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
}

// Operand entry k of row i: M[i + k ld] (ROWS_OF_COLMAJOR: the rows of a
// column-major matrix, A) or M[k + i ld] (its columns, B); tri 1 keeps only
// k <= i (A lower triangular), 2 only k >= i (B lower triangular); rows >=
// rows and k >= K are zero.
template <bool ROWS_OF_COLMAJOR, class T>
__device__ __forceinline__ double gz_at(const T *__restrict__ M, int64_t ld, int64_t rows, int64_t K, int tri,
                                        int64_t i, int64_t k) {
    if (i >= rows || k >= K) return 0.0;
    if ((tri == 1 && k > i) || (tri == 2 && k < i)) return 0.0;
    return (double)(ROWS_OF_COLMAJOR ? M[i + k * ld] : M[k + i * ld]);
}

// Pass 1: each row's max |entry| over a chunk of 1024 k (16 rows x 1024 k per
// workgroup, grid = row blocks x chunks), combined across chunks by a 64-bit
// atomic max on the (non-negative) double's bits.  rmax zeroed beforehand.
template <bool ROWS_OF_COLMAJOR, class T>
__global__ __launch_bounds__(256) void gz_max_kernel(const T *__restrict__ M, int64_t ld, int64_t rows,
                                                     int64_t K, int tri, unsigned long long *__restrict__ rmax) {
    __shared__ double red[4][16];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if constexpr (!ROWS_OF_COLMAJOR) {
        // columns of M (k contiguous): each wave reads 4 of the 16 rows, a
        // row's 1024 k as 16 coalesced 512-B wave loads
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t i = (int64_t)blockIdx.x * 16 + 4 * wave + q;
            double amax = 0.0;
#pragma unroll
            for (int c = 0; c < 16; ++c)
                amax = fmax(amax, fabs(gz_at<false>(M, ld, rows, K, tri, i, (int64_t)blockIdx.y * 1024 + 64 * c + lane)));
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) amax = fmax(amax, __shfl_xor(amax, o));
            if (lane == 0 && i < rows && amax > 0.0)
                atomicMax(rmax + i, (unsigned long long)__double_as_longlong(amax));
        }
        return;
    }
    const int r = lane & 15, g = lane >> 4;
    const int64_t i = (int64_t)blockIdx.x * 16 + r;
    const int64_t k0 = (int64_t)blockIdx.y * 1024 + wave * 256 + g * 16;
    double amax = 0.0;
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int jj = 0; jj < 16; ++jj)
            amax = fmax(amax, fabs(gz_at<ROWS_OF_COLMAJOR>(M, ld, rows, K, tri, i, k0 + 64 * c + jj)));
    amax = fmax(amax, __shfl_xor(amax, 16));
    amax = fmax(amax, __shfl_xor(amax, 32));
    if (g == 0) red[wave][r] = amax;
    __syncthreads();
    if (wave == 0 && g == 0 && i < rows) {
        amax = fmax(fmax(red[0][r], red[1][r]), fmax(red[2][r], red[3][r]));
        if (amax > 0.0) atomicMax(rmax + i, (unsigned long long)__double_as_longlong(amax));
    }
}

// Pass 1 for the Cholesky's f32 panel (the rows of a column-major m x K
// matrix): one thread per row and 128 k per workgroup, so a wave's loads are
// 64 consecutive rows (256 B) of one column -- the 16-row form above reads
// 64-B pieces and was latency-bound there (~35 us per C4 panel).
// (the f64 operands of the inverse's products too, tri as gz_at's: 1 keeps
// k <= i, 2 keeps k >= i)
template <class T>
__global__ __launch_bounds__(256) void gz_rowmax_kernel(const T *__restrict__ M, int64_t ld, int64_t rows, int64_t K,
                                                        int tri, unsigned long long *__restrict__ rmax) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= rows) return;
    int64_t k0 = (int64_t)blockIdx.y * 128, k1 = min(K, k0 + 128);
    if (tri == 1) k1 = min(k1, i + 1);
    if (tri == 2) k0 = max(k0, i);
    const T *p = M + i;
    double amax = 0.0;
#pragma unroll 16
    for (int64_t k = k0; k < k1; ++k) amax = fmax(amax, fabs((double)p[k * ld]));
    if (amax > 0.0) atomicMax(rmax + i, (unsigned long long)__double_as_longlong(amax));
}

// Pass 2: the digits, 16 rows x 4 k-blocks per workgroup (one per wave; grid
// = row blocks x ceil(Kb / 4)); thread (r, g) cuts row r's k = 16 g .. 16 g +
// 15 of its k-block into ND bytes each and stores them as one 16-B word per
// digit.  ex[i]: the row's exponent (-900: an all-zero row).
template <int ND, bool ROWS_OF_COLMAJOR, class T>
__global__ __launch_bounds__(256) void gz_digits_kernel(const T *__restrict__ M, int64_t ld, int64_t rows,
                                                        int64_t K, int Kb, int tri,
                                                        const unsigned long long *__restrict__ rmax,
                                                        char *__restrict__ out, int *__restrict__ ex) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 15, g = lane >> 4;
    const int64_t rb = blockIdx.x;
    const int64_t i = rb * 16 + r;
    const int kb = (int)blockIdx.y * 4 + wave;
    const double amax = i < rows ? __longlong_as_double((long long)rmax[i]) : 0.0;
    int e = -900;
    if (amax > 0.0) (void)frexp(amax * 1.01, &e);   // 2^e > 1.01 max: |a| 2^-e < 0.99
    if (blockIdx.y == 0 && wave == 0 && g == 0) ex[i] = e;
    constexpr int kBits = 8 * ND - 1;
    // the bias: 0x80 in each of the ND - 1 lower bytes
    constexpr int64_t kBias = (int64_t)(((uint64_t)1 << (8 * (ND - 1))) - 1) / 255 * 128;
    uint32_t w[ND][4];
    // x = rint(a 2^(kBits - e)) by ONE f64 FMA (round 6; was ldexp + rint +
    // an f64 -> i64 conversion sequence per value): fma(a, 2^(kBits - e),
    // 1.5 2^52) rounds once, to the nearest integer with ties to even (|x| <
    // 2^47 and the sum lies in [2^52, 2^53): ulp 1, and 1.5 2^52 is even); its
    // bit pattern is 0x4338000000000000 + x.  Bitwise the same digits.
    static_assert(8 * ND - 1 <= 50, "the FMA rounding needs |x| < 2^51");
    const double scale = e > -900 ? ldexp(1.0, kBits - e) : 0.0;   // (an all-zero row: x = 0)
    constexpr double kMagic = 6755399441055744.0;                 // 1.5 2^52
    // columns of M (k contiguous): the workgroup's 16 rows x 256 k staged
    // through LDS by coalesced wave loads (a row per wave load, rows padded
    // to 257 doubles), then read back in the digit order
    __shared__ double stage[ROWS_OF_COLMAJOR ? 1 : 16 * 257];
    if constexpr (!ROWS_OF_COLMAJOR) {
        const int64_t kbase = (int64_t)blockIdx.y * 4 * kGzBK;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int rr = 4 * wave + q;
#pragma unroll
            for (int c = 0; c < 4; ++c)
                stage[rr * 257 + 64 * c + lane] = gz_at<false>(M, ld, rows, K, tri, rb * 16 + rr, kbase + 64 * c + lane);
        }
    }
    __syncthreads();
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) {
        const double a = ROWS_OF_COLMAJOR
                             ? gz_at<true>(M, ld, rows, K, tri, i, (int64_t)kb * kGzBK + 16 * g + jj)
                             : stage[r * 257 + 64 * wave + 16 * g + jj];
        const uint64_t y = (uint64_t)__double_as_longlong(fma(a, scale, kMagic)) - 0x4338000000000000ull +
                           (uint64_t)kBias;
#pragma unroll
        for (int s = 0; s < ND; ++s) {
            const uint32_t b = (uint32_t)(y >> (8 * (ND - 1 - s))) & 0xFFu;
            const uint32_t d = s == 0 ? b : (b ^ 0x80u);
            if ((jj & 3) == 0) w[s][jj >> 2] = d;
            else w[s][jj >> 2] |= d << (8 * (jj & 3));
        }
    }
    if (kb >= Kb) return;
    char *base = out + ((rb * Kb + kb) * ND) * 1024 + lane * 16;
#pragma unroll
    for (int s = 0; s < ND; ++s)
        *reinterpret_cast<uint4 *>(base + s * 1024) = make_uint4(w[s][0], w[s][1], w[s][2], w[s][3]);
}

// C (m x n, ldc; transposed into C^T's storage with kGzTransC) = alpha op(A)
// op(B) (+ C with kGzBeta1) from the packed operands (op(A)'s rows, op(B)'s
// columns, Kb k-blocks each).  kGzTriA: op(A) lower triangular (a tile's k
// loop stops after its last row's diagonal block); kGzTriBLower / Upper:
// op(B) lower / upper triangular (the loop starts at the tile's first column's
// diagonal block / stops after its last column's).
template <int ND>
__global__ __launch_bounds__(256, 1) void gz_gemm_kernel(const char *__restrict__ Ad, const int *__restrict__ eA,
                                                         const char *__restrict__ Bd, const int *__restrict__ eB,
                                                         int64_t m, int64_t n, int Kb, int tilesM, double *__restrict__ C,
                                                         int64_t ldc, double alpha, unsigned flags) {
    const bool triA = flags & kGzTriA, beta1 = flags & kGzBeta1, transC = flags & kGzTransC;
    constexpr int kPieces = (kGzTM / 16 + kGzTN / 16) * ND;   // 1 KiB pieces per stage
    constexpr int kStage = kPieces * 1024;
    __shared__ __attribute__((aligned(16))) char smem[2 * kStage];
    // consecutive workgroups walk down a column of tiles (B's columns stay in
    // L2 across them); the XCD round robin spreads each column over the XCDs.
    // (Longest tiles first for a triangular A measured slower: 7.3 -> 9.3 ms
    // at 8192^3.)
    // An upper-triangular op(B): its longest columns (the last) first
    const int tilesN = (int)(gridDim.x / tilesM);
    const int tm = blockIdx.x % tilesM;
    const int tn = (flags & kGzTriBUpper) ? tilesN - 1 - (int)(blockIdx.x / tilesM) : (int)(blockIdx.x / tilesM);
    const int64_t i0 = (int64_t)tm * kGzTM, j0 = (int64_t)tn * kGzTN;
    int kb0 = 0, kb1 = Kb;
    if (flags & kGzTriBLower) kb0 = (int)(j0 / kGzBK);
    if (flags & kGzTriBUpper) kb1 = min(Kb, (int)((j0 + kGzTN - 1) / kGzBK) + 1);
    if (triA) kb1 = min(kb1, (int)((i0 + kGzTM - 1) / kGzBK) + 1);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wave_u = __builtin_amdgcn_readfirstlane(wave);

    typedef __attribute__((address_space(3))) char lds_char;
    const uint32_t lds_smem = (uint32_t)(uintptr_t)(lds_char *)(smem);
    const char *gA = Ad + (i0 / 16) * (int64_t)Kb * ND * 1024 + lane * 16;
    const char *gB = Bd + (j0 / 16) * (int64_t)Kb * ND * 1024 + lane * 16;
#define SBO_GZ_DMA16(gsrc, ldst)                                                                         \
    do {                                                                                                 \
        uint32_t keep_;                                                                                  \
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t" \
                     "s_mov_b32 m0, %0"                                                                  \
                     : "=&s"(keep_)                                                                      \
                     : "v"(gsrc), "s"(ldst)                                                              \
                     : "memory");                                                                        \
    } while (0)
    // stage k-block kb_ into buffer buf_: piece p = wave + 4 q; A's pieces
    // first (row block p / ND, digit p % ND), then B's
    auto stage = [&](int kb_, int buf_) {
#pragma unroll
        for (int q = 0; q < kPieces / 4; ++q) {
            const int p = wave_u + 4 * q;
            const int pa = p < (kGzTM / 16) * ND ? p : p - (kGzTM / 16) * ND;
            const int blk = pa / ND, s = pa % ND;
            const char *src = (p < (kGzTM / 16) * ND ? gA : gB) + ((int64_t)blk * Kb + kb_) * ND * 1024 + s * 1024;
            const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_smem + (uint32_t)(buf_ * kStage + p * 1024));
            SBO_GZ_DMA16(src, dst);
        }
    };
    static_assert(kPieces % 4 == 0, "whole pieces per wave");

    i32x4 acc[2][kGzTN / 16][ND];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int c = 0; c < kGzTN / 16; ++c)
#pragma unroll
            for (int L = 0; L < ND; ++L) acc[a][c][L] = i32x4{0, 0, 0, 0};

    if (kb0 < kb1) {
        stage(kb0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    int cur = 0;
    for (int kb = kb0; kb < kb1; ++kb) {
        if (kb + 1 < kb1) stage(kb + 1, cur ^ 1);
        const i32x4 *sA = reinterpret_cast<const i32x4 *>(smem + cur * kStage) + lane;
        const i32x4 *sB = sA + (kGzTM / 16) * ND * 64;
        i32x4 ad[2][ND];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int s = 0; s < ND; ++s) ad[a][s] = sA[((2 * wave + a) * ND + s) * 64];
#pragma unroll
        for (int c = 0; c < kGzTN / 16; ++c) {
            i32x4 bd[ND];
#pragma unroll
            for (int u = 0; u < ND; ++u) bd[u] = sB[(c * ND + u) * 64];
#pragma unroll
            for (int u = 0; u < ND; ++u)
#pragma unroll
                for (int s = 0; s + u < ND; ++s)
#pragma unroll
                    for (int a = 0; a < 2; ++a) acc[a][c][s + u] = mfma_i8(ad[a][s], bd[u], acc[a][c][s + u]);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        cur ^= 1;
    }
#undef SBO_GZ_DMA16
    // combine: lane l holds rows 4 (l >> 4) + v of each A block, column l & 15
    // of each B block
    const int g = lane >> 4, cl = lane & 15;
#pragma unroll
    for (int c = 0; c < kGzTN / 16; ++c) {
        const int64_t j = j0 + 16 * c + cl;
        if (j >= n) continue;
        const int ej = eB[j];
#pragma unroll
        for (int a = 0; a < 2; ++a) {
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int64_t i = i0 + 32 * wave + 16 * a + 4 * g + v;
                if (i >= m) continue;
                double t = (double)acc[a][c][ND - 1][v];
#pragma unroll
                for (int L = ND - 2; L >= 0; --L)
                    t = fma((double)acc[a][c][L][v], ldexp(1.0, 8 * (ND - 1 - L)), t);
                const double val = alpha * ldexp(t, eA[i] + ej - 8 * ND - 6);
                double *dst = transC ? C + j + i * ldc : C + i + j * ldc;
                *dst = beta1 ? *dst + val : val;
            }
        }
    }
}

// Round 5: the same product with more waves per SIMD -- NW = 16 (the
// default): sixteen waves of 16 x 32 (one A block and two B blocks each,
// ND x 2 int32 accumulator blocks, 95 VGPRs, four waves per SIMD); NW = 8
// (built with SBO_GZ_8WAVE): eight of 16 x 64 -- so that one wave's products
// run while the others wait on their LDS reads or the stage barrier; the
// stage and its 1 KiB LDS-DMA pieces are the four-wave kernel's.  The inverse's
// top-level products at 8192^3 (tools/ozgemm_bench.hip, packs included,
// profiles/r5_ozgemm_waves.log): 5.93 / 5.88 ms with four waves (one per
// SIMD), 5.00 / 5.06 with eight, 4.68 / 4.73 with sixteen.  Bitwise the
// four-wave kernel's results (the int32 level sums are exact in any order;
// the combination is the same code).
template <int ND, int NW, class TO, int TN = kGzTN>
__global__ __launch_bounds__(64 * NW, 1) void gz_gemm8_kernel(const char *__restrict__ Ad, const int *__restrict__ eA,
                                                              const char *__restrict__ Bd, const int *__restrict__ eB,
                                                              int64_t m, int64_t n, int Kb, int tilesM,
                                                              TO *__restrict__ C, int64_t ldc, double alpha,
                                                              unsigned flags) {
    // NW = 8: wave w = A block w, all TN / 16 B blocks; NW = 16: A block
    // w & 7, half of them (TN = 64: two; 128: four)
    constexpr int kBW = (TN / 16) * 8 / NW;      // B blocks per wave
    const bool triA = flags & kGzTriA, beta1 = flags & kGzBeta1, transC = flags & kGzTransC;
    constexpr int kPieces = (kGzTM / 16 + TN / 16) * ND;      // 1 KiB pieces per stage
    constexpr int kStage = kPieces * 1024;
    constexpr int kPerWave = (kPieces + NW - 1) / NW;
    __shared__ __attribute__((aligned(16))) char smem[2 * kStage];
    const int tilesN = (int)(gridDim.x / tilesM);
    const int tm = blockIdx.x % tilesM;
    const int tn = (flags & kGzTriBUpper) ? tilesN - 1 - (int)(blockIdx.x / tilesM) : (int)(blockIdx.x / tilesM);
    const int64_t i0 = (int64_t)tm * kGzTM, j0 = (int64_t)tn * TN;
    int kb0 = 0, kb1 = Kb;
    if (flags & kGzTriBLower) kb0 = (int)(j0 / kGzBK);
    if (flags & kGzTriBUpper) kb1 = min(Kb, (int)((j0 + TN - 1) / kGzBK) + 1);
    if (triA) kb1 = min(kb1, (int)((i0 + kGzTM - 1) / kGzBK) + 1);
    // kGzLowerC: only C's lower triangle is wanted -- a tile wholly above the
    // diagonal does nothing (the diagonal tiles are written whole)
    if ((flags & kGzLowerC) && i0 + kGzTM - 1 < j0) return;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wa = wave & 7, wb0 = (wave >> 3) * kBW;

    typedef __attribute__((address_space(3))) char lds_char;
    const uint32_t lds_smem = (uint32_t)(uintptr_t)(lds_char *)(smem);
    const char *gA = Ad + (i0 / 16) * (int64_t)Kb * ND * 1024 + lane * 16;
    const char *gB = Bd + (j0 / 16) * (int64_t)Kb * ND * 1024 + lane * 16;
#define SBO_GZ_DMA16(gsrc, ldst)                                                                         \
    do {                                                                                                 \
        uint32_t keep_;                                                                                  \
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t" \
                     "s_mov_b32 m0, %0"                                                                  \
                     : "=&s"(keep_)                                                                      \
                     : "v"(gsrc), "s"(ldst)                                                              \
                     : "memory");                                                                        \
    } while (0)
    auto stage = [&](int kb_, int buf_) {
#pragma unroll
        for (int q = 0; q < kPerWave; ++q) {
            const int p = wave + NW * q;
            if (kPieces % NW != 0 && p >= kPieces) break;   // (uniform per wave)
            const int pa = p < (kGzTM / 16) * ND ? p : p - (kGzTM / 16) * ND;
            const int blk = pa / ND, s = pa % ND;
            const char *src = (p < (kGzTM / 16) * ND ? gA : gB) + ((int64_t)blk * Kb + kb_) * ND * 1024 + s * 1024;
            const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_smem + (uint32_t)(buf_ * kStage + p * 1024));
            SBO_GZ_DMA16(src, dst);
        }
    };

    i32x4 acc[kBW][ND];
#pragma unroll
    for (int c = 0; c < kBW; ++c)
#pragma unroll
        for (int L = 0; L < ND; ++L) acc[c][L] = i32x4{0, 0, 0, 0};

    if (kb0 < kb1) {
        stage(kb0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    int cur = 0;
    for (int kb = kb0; kb < kb1; ++kb) {
        if (kb + 1 < kb1) stage(kb + 1, cur ^ 1);
        const i32x4 *sA = reinterpret_cast<const i32x4 *>(smem + cur * kStage) + lane;
        const i32x4 *sB = sA + (kGzTM / 16) * ND * 64;
        i32x4 ad[ND];
#pragma unroll
        for (int s = 0; s < ND; ++s) ad[s] = sA[(wa * ND + s) * 64];
#pragma unroll
        for (int c = 0; c < kBW; ++c) {
            i32x4 bd[ND];
#pragma unroll
            for (int u = 0; u < ND; ++u) bd[u] = sB[((wb0 + c) * ND + u) * 64];
#pragma unroll
            for (int u = 0; u < ND; ++u)
#pragma unroll
                for (int s = 0; s + u < ND; ++s) acc[c][s + u] = mfma_i8(ad[s], bd[u], acc[c][s + u]);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        cur ^= 1;
    }
#undef SBO_GZ_DMA16
    const int g = lane >> 4, cl = lane & 15;
#pragma unroll
    for (int c = 0; c < kBW; ++c) {
        const int64_t j = j0 + 16 * (wb0 + c) + cl;
        if (j >= n) continue;
        const int ej = eB[j];
        const int64_t ib = i0 + 16 * wa + 4 * g;   // the lane's four consecutive rows of column j
        if constexpr (std::is_same_v<TO, float>) {
            // (kGzVec4: C 16-B aligned with ldc % 4 == 0 -- the four rows in one
            // 16-B load and store; 16 lanes of a quarter cover a column's 64 B)
            if ((flags & kGzVec4) && !transC && ib + 3 < m) {
                f32x4v *dst = reinterpret_cast<f32x4v *>(C + ib + j * ldc);
                f32x4v o = beta1 ? *dst : f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    double t = (double)acc[c][ND - 1][v];
#pragma unroll
                    for (int L = ND - 2; L >= 0; --L) t = fma((double)acc[c][L][v], ldexp(1.0, 8 * (ND - 1 - L)), t);
                    o[v] = (float)((double)o[v] + alpha * ldexp(t, eA[ib + v] + ej - 8 * ND - 6));
                }
                *dst = o;
                continue;
            }
        }
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int64_t i = ib + v;
            if (i >= m) continue;
            double t = (double)acc[c][ND - 1][v];
#pragma unroll
            for (int L = ND - 2; L >= 0; --L) t = fma((double)acc[c][L][v], ldexp(1.0, 8 * (ND - 1 - L)), t);
            const double val = alpha * ldexp(t, eA[i] + ej - 8 * ND - 6);
            TO *dst = transC ? C + j + i * ldc : C + i + j * ldc;
            *dst = (TO)(beta1 ? (double)*dst + val : val);
        }
    }
}

template <int ND, class TI, class TO>
hipError_t gz_run(hipStream_t s, const TI *A, int64_t lda, const TI *B, int64_t ldb, int64_t m, int64_t n,
                  int64_t K, double alpha, TO *C, int64_t ldc, unsigned flags, char *ws) {
    const int Kb = (int)((K + kGzBK - 1) / kGzBK);
    const int64_t mp = (m + kGzTM - 1) / kGzTM * kGzTM, np = (n + kGzNPad - 1) / kGzNPad * kGzNPad;
    char *pa = ws;
    char *pb = pa + mp * (int64_t)Kb * kGzBK * ND;
    unsigned long long *ma = reinterpret_cast<unsigned long long *>(pb + np * (int64_t)Kb * kGzBK * ND);
    unsigned long long *mb = ma + mp;
    int *ea = reinterpret_cast<int *>(mb + np);
    int *eb = ea + mp;
    hipError_t err = hipMemsetAsync(ma, 0, sizeof(unsigned long long) * (size_t)(mp + np), s);
    if (err != hipSuccess) return err;
    const unsigned chunks = (unsigned)((K + 1023) / 1024), kq = (unsigned)((Kb + 3) / 4);
    // the rows of op(A) and the columns of op(B): rows of a column-major
    // matrix (strided k) or its columns (contiguous k); pack masks 1: k <= row,
    // 2: k >= row
    const int ta = (flags & kGzTriA) ? 1 : 0;
    const int tb = (flags & kGzTriBLower) ? 2 : (flags & kGzTriBUpper) ? 1 : 0;
    const dim3 ga((unsigned)(mp / 16), chunks), gb((unsigned)(np / 16), chunks);
    const dim3 da((unsigned)(mp / 16), kq), db((unsigned)(np / 16), kq);
    const dim3 rga((unsigned)((m + 255) / 256), (unsigned)((K + 127) / 128)),
        rgb((unsigned)((n + 255) / 256), (unsigned)((K + 127) / 128));
    if (flags & kGzTransA) {
        hipLaunchKernelGGL((gz_max_kernel<false, TI>), ga, dim3(256), 0, s, A, lda, m, K, ta, ma);
        hipLaunchKernelGGL((gz_digits_kernel<ND, false, TI>), da, dim3(256), 0, s, A, lda, m, K, Kb, ta, ma, pa, ea);
    } else {
        hipLaunchKernelGGL(gz_rowmax_kernel<TI>, rga, dim3(256), 0, s, A, lda, m, K, ta, ma);
        hipLaunchKernelGGL((gz_digits_kernel<ND, true, TI>), da, dim3(256), 0, s, A, lda, m, K, Kb, ta, ma, pa, ea);
    }
    if (flags & kGzTransB) {
        hipLaunchKernelGGL(gz_rowmax_kernel<TI>, rgb, dim3(256), 0, s, B, ldb, n, K, tb, mb);
        hipLaunchKernelGGL((gz_digits_kernel<ND, true, TI>), db, dim3(256), 0, s, B, ldb, n, K, Kb, tb, mb, pb, eb);
    } else {
        hipLaunchKernelGGL((gz_max_kernel<false, TI>), gb, dim3(256), 0, s, B, ldb, n, K, tb, mb);
        hipLaunchKernelGGL((gz_digits_kernel<ND, false, TI>), db, dim3(256), 0, s, B, ldb, n, K, Kb, tb, mb, pb, eb);
    }
    // 128-column tiles where two stages of them fit the LDS (<= 5 digits:
    // 2 x 80 KiB): twice the products per staged A block
    constexpr int TNr = ND <= 5 ? 128 : kGzTN;
    const int tilesM = (int)(mp / kGzTM), tilesN = (int)(np / TNr);
#ifdef SBO_GZ_4WAVE
    if constexpr (std::is_same_v<TO, double>) {
        if (flags & kGzLowerC) return hipErrorInvalidValue;
        hipLaunchKernelGGL((gz_gemm_kernel<ND>), dim3((unsigned)(tilesM * tilesN)), dim3(256), 0, s, pa, ea, pb, eb,
                           m, n, Kb, tilesM, C, ldc, alpha, flags);
        return hipGetLastError();
    }
#endif
#ifdef SBO_GZ_8WAVE
    hipLaunchKernelGGL((gz_gemm8_kernel<ND, 8, TO>), dim3((unsigned)(tilesM * tilesN)), dim3(512), 0, s, pa, ea, pb,
                       eb, m, n, Kb, tilesM, C, ldc, alpha, flags);
#else
    hipLaunchKernelGGL((gz_gemm8_kernel<ND, 16, TO, TNr>), dim3((unsigned)(tilesM * tilesN)), dim3(1024), 0, s, pa,
                       ea, pb, eb, m, n, Kb, tilesM, C, ldc, alpha, flags);
#endif
    return hipGetLastError();
}

}  // namespace

size_t gz_workspace_bytes(int64_t m, int64_t n, int64_t K, int nd) {
    const int64_t Kp = (K + kGzBK - 1) / kGzBK * kGzBK;
    const int64_t mp = (m + kGzTM - 1) / kGzTM * kGzTM, np = (n + kGzNPad - 1) / kGzNPad * kGzNPad;
    return (size_t)((mp + np) * Kp * nd + 12 * (mp + np)) + 256;
}

hipError_t launch_gz_gemm(hipStream_t s, int nd, const double *A, int64_t lda, const double *B, int64_t ldb,
                          int64_t m, int64_t n, int64_t K, double alpha, double *C, int64_t ldc, unsigned flags,
                          char *ws) {
    if (m <= 0 || n <= 0) return hipSuccess;
    if (K <= 0 || K > kGzMaxK) return hipErrorInvalidValue;
    if (flags & kGzLowerC) return hipErrorInvalidValue;
    switch (nd) {
        case 4: return gz_run<4>(s, A, lda, B, ldb, m, n, K, alpha, C, ldc, flags, ws);
        case 5: return gz_run<5>(s, A, lda, B, ldb, m, n, K, alpha, C, ldc, flags, ws);
        case 6: return gz_run<6>(s, A, lda, B, ldb, m, n, K, alpha, C, ldc, flags, ws);
        default: return hipErrorInvalidValue;
    }
}

// The Cholesky's panel packed once (rows padded to 128: digits, then the
// row exponents, then the row maxima) and its products read from the pack:
// op(A) = rows a0 .. a0 + m of the pack, op(B)^T = rows b0 .. b0 + n (a0, b0
// multiples of 128), K = the pack's.
size_t gz_pack_bytes(int64_t m, int64_t K, int nd) {
    const int64_t mp = (m + kGzTM - 1) / kGzTM * kGzTM, Kp = (K + kGzBK - 1) / kGzBK * kGzBK;
    return (size_t)(mp * Kp * nd + 12 * mp) + 256;
}

hipError_t launch_gz_pack_f32(hipStream_t s, int nd, const float *P, int64_t ld, int64_t m, int64_t K, char *pack) {
    if (m <= 0 || K <= 0 || K > kGzMaxK || (nd != 4 && nd != 5)) return hipErrorInvalidValue;
    const int Kb = (int)((K + kGzBK - 1) / kGzBK);
    const int64_t mp = (m + kGzTM - 1) / kGzTM * kGzTM;
    char *pd = pack;
    int *ex = reinterpret_cast<int *>(pd + mp * (int64_t)Kb * kGzBK * nd);
    unsigned long long *mx = reinterpret_cast<unsigned long long *>(
        pd + mp * (int64_t)Kb * kGzBK * nd + ((sizeof(int) * mp + 7) / 8) * 8);
    hipError_t err = hipMemsetAsync(mx, 0, sizeof(unsigned long long) * (size_t)mp, s);
    if (err != hipSuccess) return err;
    const dim3 ga((unsigned)(mp / 16), (unsigned)((K + 1023) / 1024)), da((unsigned)(mp / 16), (unsigned)((Kb + 3) / 4));
    (void)ga;
    hipLaunchKernelGGL(gz_rowmax_kernel<float>, dim3((unsigned)((m + 255) / 256), (unsigned)((K + 127) / 128)),
                       dim3(256), 0, s, P, ld, m, K, 0, mx);
    if (nd == 4)
        hipLaunchKernelGGL((gz_digits_kernel<4, true, float>), da, dim3(256), 0, s, P, ld, m, K, Kb, 0, mx, pd, ex);
    else
        hipLaunchKernelGGL((gz_digits_kernel<5, true, float>), da, dim3(256), 0, s, P, ld, m, K, Kb, 0, mx, pd, ex);
    return hipGetLastError();
}

hipError_t launch_gz_gemm_packed_f32(hipStream_t s, int nd, const char *pack, int64_t mpack, int64_t K, int64_t a0,
                                     int64_t m, int64_t b0, int64_t n, double alpha, float *C, int64_t ldc,
                                     unsigned flags) {
    if (m <= 0 || n <= 0) return hipSuccess;
    if (K <= 0 || K > kGzMaxK || (nd != 4 && nd != 5) || a0 % kGzTM != 0 || b0 % kGzTM != 0 || a0 + m > mpack ||
        b0 + n > mpack || (flags & (kGzTransC | kGzTriA | kGzTriBLower | kGzTriBUpper)))
        return hipErrorInvalidValue;
    const int Kb = (int)((K + kGzBK - 1) / kGzBK);
    const int64_t mp = (mpack + kGzTM - 1) / kGzTM * kGzTM;
    const int *ex = reinterpret_cast<const int *>(pack + mp * (int64_t)Kb * kGzBK * nd);
    const int64_t blk = (int64_t)Kb * nd * 1024;   // one 16-row block of the pack
    const char *pa = pack + (a0 / 16) * blk, *pb = pack + (b0 / 16) * blk;
    // 128 x 128 tiles (four B blocks per wave): twice the products per
    // staged k-block and per prologue / epilogue of the short k = 512 loop
    // (two 64 / 80 KiB stages fit the LDS at 4 / 5 digits)
    constexpr int TN = 128;
    const int tilesM = (int)((m + kGzTM - 1) / kGzTM), tilesN = (int)((n + TN - 1) / TN);
    if (b0 + (n + TN - 1) / TN * TN > (mpack + kGzTM - 1) / kGzTM * kGzTM) return hipErrorInvalidValue;
    if (((uintptr_t)C % 16) == 0 && ldc % 4 == 0) flags |= kGzVec4;
    if (nd == 4)
        hipLaunchKernelGGL((gz_gemm8_kernel<4, 16, float, TN>), dim3((unsigned)(tilesM * tilesN)), dim3(1024), 0, s,
                           pa, ex + a0, pb, ex + b0, m, n, Kb, tilesM, C, ldc, alpha, flags);
    else
        hipLaunchKernelGGL((gz_gemm8_kernel<5, 16, float, TN>), dim3((unsigned)(tilesM * tilesN)), dim3(1024), 0, s,
                           pa, ex + a0, pb, ex + b0, m, n, Kb, tilesM, C, ldc, alpha, flags);
    return hipGetLastError();
}

hipError_t launch_gz_gemm_f32(hipStream_t s, int nd, const float *A, int64_t lda, const float *B, int64_t ldb,
                              int64_t m, int64_t n, int64_t K, double alpha, float *C, int64_t ldc, unsigned flags,
                              char *ws) {
    if (m <= 0 || n <= 0) return hipSuccess;
    if (K <= 0 || K > kGzMaxK) return hipErrorInvalidValue;
    if ((flags & kGzLowerC) && (flags & kGzTransC)) return hipErrorInvalidValue;
    switch (nd) {
        case 4: return gz_run<4>(s, A, lda, B, ldb, m, n, K, alpha, C, ldc, flags, ws);
        case 5: return gz_run<5>(s, A, lda, B, ldb, m, n, K, alpha, C, ldc, flags, ws);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace sbo
