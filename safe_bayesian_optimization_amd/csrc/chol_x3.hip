// chol_x3.hip -- the blocked Cholesky's rank-512 updates (a2) on the bf16
// matrix cores with split operands (round 5, SBO_OPT_CHOL_GEMM 3).
//
// The factorization's flops are its outer panels' updates C -= P P^T (the
// look-ahead block column and the lower trailing triangle, k = 512): rocBLAS
// sgemm / ssyrk and the library's own f32-MFMA chol_update_kernel ran them at
// 55-97 TF against the 157 TF f32 matrix peak (profiles/r3_update_probe.log),
// 19.2 ms of the C4 fit's 45 ms (profiles/r4_fit_c4_trace_oz.txt).  As in the
// predictive sweep (predict_x3.hip), every f32 operand value is split into
// three bf16 pieces, v = v0 + v1 + v2 (round to nearest at each step), and a
// product is the six terms a2 b0 + a1 b1 + a0 b2 + a1 b0 + a0 b1 + a0 b0 (the
// dropped ones below 2^-23 |a b|, the order of an f32 rounding), each one
// v_mfma_f32_16x16x32_bf16 with f32 accumulation: 6 x 16 cycles per 16x16x32
// block against 8 x 32 for v_mfma_f32_16x16x4_f32.
//
//   chol_split_kernel: the outer panel (m x K f32, column-major) once into the
//     three planes in MFMA fragment order -- [32-k chunk][16-row block][plane]
//     [lane][16 B], lane l holding row 16 b + (l & 15), k 32 c + 8 (l >> 4) ..
//     + 7 -- so that a 16-row block of a chunk is 3 KiB contiguous and a
//     lane's MFMA operand is one ds_read_b128 (K = 512: 6 B per element, 48 MB
//     at m = 16384, double-buffered across outer panels by the caller);
//   chol_update_x3_kernel: C (rows x cols, lda ld, relative to the region's
//     origin) -= P Q^T with P the panel's rows r0 .. and Q its rows c0 .. --
//     256 x 128 tiles of C (lower: the tiles that meet the lower triangle of a
//     square region), eight waves of 64 x 64, the planes of both operands
//     staged 32 k at a time by LDS-DMA (72 KiB per chunk, double buffered);
//     the MFMA's A side takes Q (C's columns) and its B side P (C's rows), so
//     a lane's four results are four columns of one C row and the 16 lanes of
//     a quarter store 64 contiguous bytes.  The accumulator starts at -C and
//     -acc is stored: C - P Q^T with one f32 rounding per MFMA step, as a
//     k-ordered accumulation (not bitwise the fmaf chain of chol_update_kernel
//     or rocBLAS: the factor differs from theirs at the f32 rounding level).
#include <cstdint>

#include "sbo_internal.hpp"

namespace sbo {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) char lds_char;

constexpr int kCxK = 32;                              // k per chunk: one 16x16x32 MFMA
constexpr int kCxBlk = 3 * 1024;                      // a 16-row block's three planes of one chunk
constexpr int kCxTR = 256, kCxTC = 128;               // workgroup tile: C rows (P) x C columns (Q)
constexpr int kCxPB = kCxTR / 16, kCxQB = kCxTC / 16; // 16 P blocks, 8 Q blocks
constexpr int kCxPBytes = kCxPB * kCxBlk;             // 48 KiB
constexpr int kCxStage = kCxPBytes + kCxQB * kCxBlk;  // 72 KiB
constexpr int kCxWaves = 8;
constexpr int kCxPieces = kCxStage / 1024 / kCxWaves; // 9 LDS-DMA pieces per wave per chunk
static_assert(kCxPieces * 1024 * kCxWaves == kCxStage, "whole pieces per wave");
static_assert(2 * kCxStage <= 160 * 1024, "two stages in the LDS");

__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
    const f32x2 v = {a, b};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
}
__device__ __forceinline__ float lo_f32(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi_f32(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

__global__ __launch_bounds__(256) void chol_split_kernel(const float *__restrict__ P, int64_t ld, int m, int nb,
                                                         int64_t units, char *__restrict__ out) {
    const int64_t u = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);   // unit = chunk * nb + block
    if (u >= units) return;
    const int lane = threadIdx.x & 63;
    const int c = (int)(u / nb), b = (int)(u % nb);
    const int row = 16 * b + (lane & 15);
    const int k0 = kCxK * c + 8 * (lane >> 4);
    const bool in = row < m;
    const float *p = P + (in ? row : 0) + (int64_t)k0 * ld;
    u32x4 w0, w1, w2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float a = in ? p[(int64_t)(2 * j) * ld] : 0.0f;
        const float bb = in ? p[(int64_t)(2 * j + 1) * ld] : 0.0f;
        const uint32_t h = pk_bf16(a, bb);
        const float ra = a - lo_f32(h), rb = bb - hi_f32(h);
        const uint32_t md = pk_bf16(ra, rb);
        w0[j] = h;
        w1[j] = md;
        w2[j] = pk_bf16(ra - lo_f32(md), rb - hi_f32(md));
    }
    char *o = out + (size_t)u * kCxBlk + lane * 16;
    *reinterpret_cast<u32x4 *>(o) = w0;
    *reinterpret_cast<u32x4 *>(o + 1024) = w1;
    *reinterpret_cast<u32x4 *>(o + 2048) = w2;
}

__device__ __forceinline__ f32x4 mfma(u32x4 a, u32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                   0, 0);
}

// tiles of a lower region: row tile i holds min(2 i + 2, ntj) column tiles
__device__ __forceinline__ void lower_tile(int q, int ntj, int &i, int &j) {
    int cum = 0, t = 0;
    for (;;) {
        const int cnt = min(2 * t + 2, ntj);
        if (q < cum + cnt) break;
        cum += cnt;
        ++t;
    }
    i = t;
    j = q - cum;
}

__global__ __launch_bounds__(512, 1) void chol_update_x3_kernel(const char *__restrict__ planes, int nb, int nch,
                                                                int rb0, int rows, int cb0, int cols, int lower,
                                                                float *__restrict__ C, int64_t ld) {
    __shared__ __attribute__((aligned(16))) char smem[2 * kCxStage];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 1, wc = wave & 1;   // the wave's 64 x 64: rows 64 wr, columns 64 wc of the tile
    int ti, tj;
    const int ntj = (cols + kCxTC - 1) / kCxTC;
    if (lower) {
        lower_tile((int)blockIdx.x, ntj, ti, tj);
    } else {
        ti = (int)blockIdx.x / ntj;
        tj = (int)blockIdx.x % ntj;
    }
    ti = __builtin_amdgcn_readfirstlane(ti);
    tj = __builtin_amdgcn_readfirstlane(tj);
    const int R0 = ti * kCxTR + 64 * wr, C0 = tj * kCxTC + 64 * wc;   // the wave's first row / column
    // the wave's region is outside C, or (lower) strictly above the diagonal
    const bool idle = R0 >= rows || C0 >= cols || (lower && R0 + 63 < C0);

    // LDS-DMA (global_load_lds_dwordx4 v_off, s_base): piece t of a chunk is
    // P's (t < 48) or Q's 1 KiB at t * 1024 of the stage; wave w moves pieces
    // w, w + 8, ..; a piece of a block past the panel moves nothing (EXEC 0)
    const uint32_t voff = (uint32_t)lane * 16u;
    const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_char *)(smem);
    const int pblk0 = rb0 + ti * kCxPB, qblk0 = cb0 + tj * kCxQB;   // first P / Q block of the tile
    auto stage = [&](int ch, int buf) {
#pragma unroll
        for (int s = 0; s < kCxPieces; ++s) {
            const int t = wave + kCxWaves * s;
            const bool isp = t < kCxPB * 3;
            const int blk = isp ? pblk0 + t / 3 : qblk0 + (t - kCxPB * 3) / 3;
            const int pl = isp ? t % 3 : (t - kCxPB * 3) % 3;
            const uint32_t m32 = (uint32_t)__builtin_amdgcn_readfirstlane(blk < nb ? -1 : 0);
            const uint64_t mask = ((uint64_t)m32 << 32) | m32;
            const uint64_t sa = (uint64_t)(uintptr_t)(planes + ((size_t)ch * nb + (size_t)(blk < nb ? blk : 0)) * kCxBlk +
                                                      pl * 1024);
            const char *src = reinterpret_cast<const char *>(
                (uintptr_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(sa >> 32)) << 32) |
                            (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)sa)));
            const uint32_t dst = lds0 + (uint32_t)(buf * kCxStage + t * 1024);
            uint64_t sv;
            asm volatile("s_mov_b64 %0, exec\n\ts_and_b64 exec, exec, %4\n\ts_nop 0\n\t"
                         "global_load_lds_dwordx4 %1, %2\n\ts_mov_b64 exec, %0"
                         : "=&s"(sv)
                         : "v"(voff), "s"((const void *)src), "{m0}"(dst), "s"(mask)
                         : "memory", "scc");
        }
    };

    // accumulators: acc[qb][pb] = -C over the wave's 4 x 4 blocks; lane l
    // holds C row R0 + 16 pb + (l & 15), columns C0 + 16 qb + 4 (l >> 4) + v
    const int fr = lane & 15, fg = lane >> 4;
    f32x4 acc[4][4];
#pragma unroll
    for (int qb = 0; qb < 4; ++qb)
#pragma unroll
        for (int pb = 0; pb < 4; ++pb) {
            const int r = R0 + 16 * pb + fr;
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int c = C0 + 16 * qb + 4 * fg + v;
                acc[qb][pb][v] = (!idle && r < rows && c < cols) ? -C[r + (int64_t)c * ld] : 0.0f;
            }
        }

    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int ch = 0; ch < nch; ++ch) {
        const int buf = ch & 1;
        if (ch + 1 < nch) stage(ch + 1, buf ^ 1);
        if (!idle) {
            const lds_char *sp = (const lds_char *)smem + buf * kCxStage + lane * 16;
            u32x4 q[4][3], p[4][3];
#pragma unroll
            for (int x = 0; x < 4; ++x)
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) {
                    q[x][pl] = *reinterpret_cast<const __attribute__((address_space(3))) u32x4 *>(
                        sp + kCxPBytes + ((4 * wc + x) * 3 + pl) * 1024);
                    p[x][pl] = *reinterpret_cast<const __attribute__((address_space(3))) u32x4 *>(
                        sp + ((4 * wr + x) * 3 + pl) * 1024);
                }
#pragma unroll
            for (int qb = 0; qb < 4; ++qb)
#pragma unroll
                for (int pb = 0; pb < 4; ++pb) {
                    f32x4 v = acc[qb][pb];
                    v = mfma(q[qb][2], p[pb][0], v);
                    v = mfma(q[qb][1], p[pb][1], v);
                    v = mfma(q[qb][0], p[pb][2], v);
                    v = mfma(q[qb][1], p[pb][0], v);
                    v = mfma(q[qb][0], p[pb][1], v);
                    v = mfma(q[qb][0], p[pb][0], v);
                    acc[qb][pb] = v;
                }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    if (idle) return;
#pragma unroll
    for (int qb = 0; qb < 4; ++qb)
#pragma unroll
        for (int pb = 0; pb < 4; ++pb) {
            const int r = R0 + 16 * pb + fr;
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int c = C0 + 16 * qb + 4 * fg + v;
                if (r < rows && c < cols) C[r + (int64_t)c * ld] = -acc[qb][pb][v];
            }
        }
}

}  // namespace

size_t chol_x3_bytes(int64_t m, int64_t K) {
    return (size_t)((m + 15) / 16) * (size_t)(K / kCxK) * (size_t)kCxBlk;
}

hipError_t launch_chol_split(hipStream_t s, const float *P, int64_t ld, int64_t m, int64_t K, char *planes) {
    if (m <= 0 || K <= 0 || K % kCxK != 0 || m > INT32_MAX / 2) return hipErrorInvalidValue;
    const int64_t nb = (m + 15) / 16, units = nb * (K / kCxK);
    hipLaunchKernelGGL(chol_split_kernel, dim3((unsigned)((units + 3) / 4)), dim3(256), 0, s, P, ld, (int)m, (int)nb,
                       units, planes);
    return hipGetLastError();
}

hipError_t launch_chol_update_x3(hipStream_t s, const char *planes, int64_t m, int64_t K, int64_t r0, int64_t rows,
                                 int64_t c0, int64_t cols, bool lower, float *C, int64_t ld) {
    // (the planes hold the panel's m rows; the regions' first rows must start
    // a 16-row block, and a lower region is square on the diagonal)
    if (m <= 0 || K <= 0 || K % kCxK != 0 || r0 < 0 || c0 < 0 || r0 % 16 != 0 || c0 % 16 != 0 || rows < 0 ||
        cols < 0 || r0 + rows > m || c0 + cols > m || (lower && (r0 != c0 || rows != cols)) || m > INT32_MAX / 2)
        return hipErrorInvalidValue;
    if (rows == 0 || cols == 0) return hipSuccess;
    const int64_t nti = (rows + kCxTR - 1) / kCxTR, ntj = (cols + kCxTC - 1) / kCxTC;
    int64_t tiles = 0;
    if (lower)
        for (int64_t i = 0; i < nti; ++i) tiles += std::min<int64_t>(2 * i + 2, ntj);
    else
        tiles = nti * ntj;
    hipLaunchKernelGGL(chol_update_x3_kernel, dim3((unsigned)tiles), dim3(512), 0, s, planes, (int)((m + 15) / 16),
                       (int)(K / kCxK), (int)(r0 / 16), (int)rows, (int)(c0 / 16), (int)cols, lower ? 1 : 0, C, ld);
    return hipGetLastError();
}

}  // namespace sbo
