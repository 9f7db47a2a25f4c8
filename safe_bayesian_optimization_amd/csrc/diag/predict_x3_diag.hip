// diag/predict_x3_diag.hip -- the split sweep with every A/B and timing
// variant of rounds 1-3 (the DIAG template mask): built only into the
// diagnostic library (make diag, -DSBO_DIAG, lib/libsbo_diag.so, selected by
// SBO_LIB for tools/).  The product sweep is ../predict_x3.hip: variant 3 of
// this file with its options fixed, one code path; variant 3 here is bitwise
// that kernel (tools/compare_libs.py).
//
// Every f32 operand value v is split into three bf16 pieces, v = v0 + v1 + v2
// (round to nearest at each step: |v1| <= 2^-8 |v|, |v2| <= 2^-16 |v|, the
// remainder below 2^-24 |v|), and a product a*k is taken as the six terms
//     a2 k0 + a1 k1 + a0 k2 + a1 k0 + a0 k1 + a0 k0
// (smallest first; the dropped a1 k2, a2 k1, a2 k2 are below 2^-23 |a k|,
// the order of an f32 rounding).  Each term is one v_mfma_f32_16x16x32_bf16
// (exact bf16 products, f32 accumulation): 6 x 16 cycles per 16x16x32
// block against 8 x 32 cycles of v_mfma_f32_16x16x4_f32, and unlike the f32
// MFMA, a bf16 MFMA leaves the SIMD's vector issue free for 8 of its 16
// cycles, so the K* chain and its split run in the matrix pipe's shadow.
//
// A = sf2 L^-1 is split once per fit/append/import (pack_x3_kernel, from the
// f32 packed operand); K* is split in registers as it is generated.
//
// Work items, the tick plan and the persistent walk are those of
// predict_kernel (kernels.hip): workgroup = 256 rows x 128 queries, eight
// waves, wave w owns queries 16w..16w+15 and all 256 rows as sixteen 16-row
// MFMA blocks; each 64-k tile is two half-steps of 32 k (an LDS stage of
// 3 planes x 256 rows x 32 k bf16 = 48 KiB), its MFMA chain starts from zero
// and is added into an f32 outer sum once the tile is done.
//
// Staging: three LDS slots, stage i+2 issued at the top of step i by LDS-DMA
// (global_load_lds_dwordx4 from inline asm), retired by a counted vmcnt at
// the end of step i+1; the slot also carries the half-tile's coordinates,
// sf2 alpha and the item's 128 query coordinates, which the first loader
// wave issues BEFORE its A pieces, so that the end-of-step wait that leaves
// the A pieces of stage i+2 in flight has retired them -- the K* of step
// i+1 is computed during step i, beside its MFMAs.
#include <cstdint>
#include <cstdlib>
#include <algorithm>
#include <type_traits>
#include <vector>

#include "../sbo_internal.hpp"

namespace sbo {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kXH = 32;                  // k per half-step
constexpr int kXPlane = kBM * kXH * 2;   // one bf16 plane of a half-tile: 16 KiB
constexpr int kXA = 3 * kXPlane;         // the A stage: 48 KiB
constexpr int kXC = 4 * kXH * 4;         // x[32], y[32], sf2 alpha[32], pad: 512 B
constexpr int kXQ = 2 * kBN * 4;         // the item's qx[128], qy[128]: 1 KiB
constexpr int kXSlot = kXA + kXC + kXQ;  // 50,688 B
constexpr int kXSlots = 3;
constexpr int kXWin = kXSlots * kXSlot;  // descriptor and tile-list windows follow the slots
constexpr int kXSmem = kXWin + 4096;
constexpr int kRecWin = 64;  // step records (int4) per 1 KiB LDS window

__device__ __forceinline__ float fast_exp2(float v) { return __builtin_amdgcn_exp2f(v); }
__device__ __forceinline__ float lo_f32(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi_f32(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// two f32 -> one dword of two bf16 (element 0 low), round to nearest even
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
    const f32x2 v = {a, b};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
}

// v = v0 + v1 + v2 for a pair of values (element 0 in the low halves)
__device__ __forceinline__ void split3(float a, float b, uint32_t &w0, uint32_t &w1, uint32_t &w2) {
    w0 = pk_bf16(a, b);
    const float ra = a - lo_f32(w0), rb = b - hi_f32(w0);
    w1 = pk_bf16(ra, rb);
    w2 = pk_bf16(ra - lo_f32(w1), rb - hi_f32(w1));
}

__device__ __forceinline__ bf16x8 as_bf16x8(u32x4 v) { return __builtin_bit_cast(bf16x8, v); }

__device__ __forceinline__ f32x4 mfma(u32x4 a, u32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(a), as_bf16x8(b), c, 0, 0, 0);
}

typedef __attribute__((address_space(3))) char lds_char;

__device__ __forceinline__ u32x4 lds_b128(const lds_char *p) {
    return *reinterpret_cast<const __attribute__((address_space(3))) u32x4 *>(p);
}
__device__ __forceinline__ float lds_f(const lds_char *p) {
    return *reinterpret_cast<const __attribute__((address_space(3))) float *>(p);
}

// One LDS-DMA piece: 64 lanes x 16 B from sbase + voff to LDS at M0 = ldst
// (+ lane x 16).  s_nop: the M0 write -> LDS-DMA hazard.
__device__ __forceinline__ void dma16(uint32_t voff, const void *sbase, uint32_t ldst) {
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "{m0}"(ldst) : "memory");
}
// the same under a wave-uniform EXEC mask (0: no lane moves data, but the
// instruction still issues and counts in vmcnt, so the step's wait count
// stays static) -- no control flow in the scheduled MFMA region
__device__ __forceinline__ void dma16_masked(uint32_t voff, const void *sbase, uint32_t ldst, uint64_t mask) {
    uint64_t sv;
    asm volatile("s_mov_b64 %0, exec\n\ts_and_b64 exec, exec, %4\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\t"
                 "s_mov_b64 exec, %0"
                 : "=&s"(sv)
                 : "v"(voff), "s"(sbase), "{m0}"(ldst), "s"(mask)
                 : "memory", "scc");
}

// K* pieces of a step for the wave's NC 16-query column blocks
// (lane (g, r): k = 8g + j of the half-tile, query 16 (NC w + c) + r)
template <int NC>
struct KPieces {
    u32x4 h[NC], m[NC], l[NC];
};

typedef float f32x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2v lds_f2(const lds_char *p) {
    return *reinterpret_cast<const __attribute__((address_space(3))) f32x2v *>(p);
}

__device__ __forceinline__ float kstar1(float xk, float yk, float xq, float yq, float cexp) {
    const float dx = xk - xq, dy = yk - yq;
    return fast_exp2(fmaf(dy, dy, dx * dx) * cexp);
}

// Pin a value's computation to this point of the instruction stream (the
// IR-level sinking passes ignore sched_barrier and would otherwise bunch the
// next step's K* work after the last MFMA), in an arch VGPR.
#define SBO_PIN(v) asm volatile("" : "+v"(v))
#ifdef SBO_X3_PIN_OUTER
#define SBO_PIN_O(v) SBO_PIN(v)
#else
#define SBO_PIN_O(v) do { } while (0)
#endif

// One half-step of one wave: 16 row blocks x NC column blocks x 6 MFMAs on
// this slot's A planes (each A fragment feeds every column block) and this
// step's K* pieces kb, with the next step's K* pieces and its mean terms
// (scaled by msc: 1 for the last row block, else 0) built beside them: pair i of every column
// block in row blocks 4i .. 4i+3 (read the pair's coordinates, evaluate,
// split and add the mean terms).
//   FRESH: first half of a tile (the chains start from zero); otherwise the
//   finished chains of each row block are added into `outer` two blocks
//   later (off the MFMA's result latency).
//   LV: the tile's precision level (the plan's code): 0 all six products,
//   1 the three largest (a1 kh + a0 km + a0 kh), 2 a0 kh alone; the A planes
//   a level leaves out are not read from LDS.
//   KHN: the next step is a one-product step too (DIAG & 1073741824 selects
//   this body then): its K* pieces are kh alone, the split is skipped (a
//   one-product step reads no other piece, so the results are bitwise those
//   of the full split).
//   MEAN: 1 the next step is the mean's row block, 0 it is not (compile
//   time: a uniform branch inside the MFMA region splits it into separately
//   scheduled pieces, four per half-step), -1 the runtime test of msc.
template <int NC, bool FRESH, long long DIAG, int PIECES, int LV = 0, bool KHN = false, int MEAN = -1>
__device__ __forceinline__ void x3_half(const lds_char *pa, const lds_char *pcn, const float (&xq)[NC],
                                        const float (&yq)[NC], int g, float cexp, float msc, const KPieces<NC> &kb,
                                        f32x4 (&acc)[NC][16], f32x4 (&outer)[NC][16], KPieces<NC> &nx,
                                        double (&mu)[NC], uint32_t voff, const char *asrc, uint32_t adst,
                                        bool loader, int npieces) {
    // SPREAD (DIAG & 16): this wave's A pieces of stage i+2 are issued one
    // per row block between the MFMAs instead of in a burst at the top
    constexpr bool SPREAD = (DIAG & 16) != 0;
    constexpr int kStride = (PIECES == 6 ? 8 : 4) * 1024;  // loader waves x 1 KiB
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
    // A fragments: row block rb in use, rb+1 landed or landing, rb+2 issued
    // during rb (DIAG & 32: one block ahead only)
    constexpr int AHEAD = (DIAG & 32) ? 1 : 2;
    // (DIAG 2048 / 4096: every tile at level 1 / 2, timing diagnostics)
    constexpr int EL = (DIAG & 4096) ? 2 : ((DIAG & 2048) ? 1 : LV);
    constexpr bool P1 = EL <= 1, P2 = EL == 0;  // planes a1, a2 in use
    constexpr int NPROD = EL == 0 ? 6 : (EL == 1 ? 3 : 1);
    // DIR: this level's products accumulate straight into the outer sums
    // (no per-tile chain, no outer add): DIAG & 2097152 one product,
    // DIAG & 4194304 three products as well
    constexpr bool DIR = (EL == 2 && (DIAG & 2097152)) || (EL == 1 && (DIAG & 4194304));
    constexpr int LAG = (DIAG & 32768) ? 2 : (EL == 0 ? 2 : (EL == 1 ? 4 : 8));
    // DIAG & 33554432: the next pair's coordinates read at ph 1 instead of ph 3
    constexpr bool EARLY_XY = (DIAG & 33554432) != 0;
    const int npu = __builtin_amdgcn_readfirstlane(npieces);
    // A fragments of row block r are read AH blocks ahead of their use: the
    // fewer MFMAs a block has, the more blocks ahead (DIAG & 65536: 4 at one
    // product, 2 at three), so the LDS latency stays covered
    constexpr int AH = (DIAG & 131072) ? (EL == 2 ? 8 : (EL == 1 ? 3 : AHEAD))
                       : (DIAG & 65536) ? (EL == 2 ? 4 : (EL == 1 ? 2 : AHEAD)) : AHEAD;
    u32x4 f0[16], f1[16], f2[16];
#pragma unroll
    for (int r = 0; r < AH; ++r) {
        f0[r] = lds_b128(pa + r * 1024);
        if constexpr (P1) f1[r] = lds_b128(pa + kXPlane + r * 1024);
        if constexpr (P2) f2[r] = lds_b128(pa + 2 * kXPlane + r * 1024);
    }
    // coordinates of pair 0; pair i+1's are read while pair i is built
    // DIAG & 67108864: sf2 alpha read only before the mean's row block (msc != 0)
    constexpr bool AK_MEAN = (DIAG & 67108864) != 0;
    f32x2v xk = lds_f2(pcn + g * 32), yk = lds_f2(pcn + 128 + g * 32), ak = {0.f, 0.f};
    if (!AK_MEAN || (MEAN < 0 ? msc != 0.0f : MEAN == 1)) ak = lds_f2(pcn + 256 + g * 32);
    f32x2v e[NC];
#pragma unroll
    for (int rb = 0; rb < 16; ++rb) {
        if (rb + AH < 16) {
            f0[rb + AH] = lds_b128(pa + (rb + AH) * 1024);
            if constexpr (P1) f1[rb + AH] = lds_b128(pa + kXPlane + (rb + AH) * 1024);
            if constexpr (P2) f2[rb + AH] = lds_b128(pa + 2 * kXPlane + (rb + AH) * 1024);
        }
        const u32x4 a0 = f0[rb];
        u32x4 a1 = {}, a2 = {};
        if constexpr (P1) a1 = f1[rb];
        if constexpr (P2) a2 = f2[rb];
        // ---- the next step's K*, pair i over row blocks 4i .. 4i+3:
        // evaluate (two slots), split, mean terms + the next pair's coordinates
        const int i = rb >> 2, ph = rb & 3;
        if (DIAG & 1) {
        } else if (ph <= 1) {
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                // (DIAG & 536870912: timing bound of a one-multiply K*, wrong results)
                float ev = (DIAG & 536870912) ? (ph == 0 ? xk.x : xk.y) * xq[c]
                                              : kstar1(ph == 0 ? xk.x : xk.y, ph == 0 ? yk.x : yk.y, xq[c], yq[c], cexp);
                SBO_PIN(ev);
                if (ph == 0) e[c].x = ev; else e[c].y = ev;
            }
            // EARLY_XY: the next pair's x, y two row blocks earlier than at ph 3
            if (EARLY_XY && ph == 1 && i < 3) {
                xk = lds_f2(pcn + g * 32 + (i + 1) * 8);
                yk = lds_f2(pcn + 128 + g * 32 + (i + 1) * 8);
            }
        } else if (ph == 2) {
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                uint32_t w0, w1, w2;
                if constexpr ((DIAG & 1048576) != 0) {  // timing diagnostic: kh only (results wrong beyond level 2)
                    w0 = pk_bf16(e[c].x, e[c].y);
                    w1 = w0;
                    w2 = w0;
                } else if constexpr (KHN) {  // the next step runs at one product: kh alone
                    w0 = pk_bf16(e[c].x, e[c].y);
                    SBO_PIN(w0);
                    nx.h[c][i] = w0;
                    continue;
                } else {
                    split3(e[c].x, e[c].y, w0, w1, w2);
                }
                SBO_PIN(w0);
                SBO_PIN(w1);
                SBO_PIN(w2);
                nx.h[c][i] = w0;
                nx.m[c][i] = w1;
                nx.l[c][i] = w2;
            }
        } else {
            // (DIAG & 2^32: the mean terms by a select, every step, instead of a branch)
            constexpr bool BLM = (DIAG & 4294967296LL) != 0;
            if constexpr (BLM) {
                const bool mn = msc != 0.0f;
#pragma unroll
                for (int c = 0; c < NC; ++c) {
                    const double t = (double)fmaf(ak.x, e[c].x, ak.y * e[c].y);
                    mu[c] = mn ? mu[c] + t : mu[c];
                    SBO_PIN(mu[c]);
                }
            } else if (MEAN < 0 ? msc != 0.0f : MEAN == 1) {  // the next step is the mean's row block
#pragma unroll
                for (int c = 0; c < NC; ++c) {
                    // the pair's terms in f32 (one rounding of a two-term sum,
                    // the order of K*'s own), accumulated in f64
                    mu[c] += (double)fmaf(ak.x, e[c].x, ak.y * e[c].y);
                    SBO_PIN(mu[c]);
                }
            }
            if (i < 3) {
                if (!EARLY_XY) {
                    xk = lds_f2(pcn + g * 32 + (i + 1) * 8);
                    yk = lds_f2(pcn + 128 + g * 32 + (i + 1) * 8);
                }
                if (!AK_MEAN || (MEAN < 0 ? msc != 0.0f : MEAN == 1)) ak = lds_f2(pcn + 256 + g * 32 + (i + 1) * 8);
            }
        }
        if (SPREAD && rb >= 1 && rb <= PIECES && loader) {
            // (DIAG & 8192: only the pieces of the planes the staged tile's level reads)
            if constexpr (DIAG & 16384) {
                // issued after the row block instead (below)
            } else if constexpr (DIAG & 8192) {
                const uint32_t mh = (uint32_t)__builtin_amdgcn_readfirstlane(rb <= npieces ? -1 : 0);
                dma16_masked(voff, asrc + (rb - 1) * kStride, adst + (rb - 1) * kStride,
                             ((uint64_t)mh << 32) | mh);
            }
            else
                dma16(voff, asrc + (rb - 1) * kStride, adst + (rb - 1) * kStride);
        }
        // the finished chains of block rb - LAG (LAG row blocks = 2 (six
        // products), 4 (three) or 8 (one) x NPROD MFMAs ago: off the MFMA
        // result latency)
        if (!FRESH && !(DIAG & 68) && !DIR && rb >= LAG) {
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                outer[c][rb - LAG] += acc[c][rb - LAG];
                SBO_PIN_O(outer[c][rb - LAG]);
            }
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            // (DIAG & 64: one chain over the whole item, no outer sums -- timing only)
            f32x4 v = DIR ? outer[c][rb] : ((FRESH && !(DIAG & 64)) ? zero : acc[c][rb]);
            if constexpr (P2) {
                v = mfma(a2, kb.h[c], v);
                v = mfma(a1, kb.m[c], v);
                v = mfma(a0, kb.l[c], v);
            }
            if constexpr (P1) {
                v = mfma(a1, kb.h[c], v);
                v = mfma(a0, kb.m[c], v);
            }
            v = mfma(a0, kb.h[c], v);
            if constexpr (DIR) outer[c][rb] = v;
            else acc[c][rb] = v;
        }
        // interleave: each MFMA followed by two VALU and one LDS read, so the
        // vector work issues in the matrix pipe's shadow (a bf16 MFMA holds
        // the SIMD's issue for 8 of its 16 cycles)
        if constexpr (DIAG & 128) {  // A/B: more VALU per MFMA gap
#pragma unroll
            for (int j = 0; j < NPROD * NC; ++j) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
                __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);  // VALU
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
            }
        } else if constexpr (!(DIAG & 256)) {  // (256: the compiler's own order)
#pragma unroll
            for (int j = 0; j < NPROD * NC; ++j) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
                __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // VALU
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        // DIAG & 16384: piece rb of stage i+2 after row block rb, and only the
        // planes its level reads (a uniform branch at the scheduling-region
        // boundary; the step's vmcnt wait counts npieces)
        if constexpr (SPREAD && (DIAG & 16384)) {
            if (rb < PIECES && loader && (rb < PIECES / 3 || rb < npu))
                dma16(voff, asrc + rb * kStride, adst + rb * kStride);
        }
    }
    if constexpr (DIR && FRESH) {
        // a tile's halves share its level: the second half of a DIR tile
        // never reads acc, so leave it undefined here (else its stale value
        // stays live through this path into the other levels' second halves)
#pragma unroll
        for (int rb = 0; rb < 16; ++rb)
#pragma unroll
            for (int c = 0; c < NC; ++c) acc[c][rb] = __builtin_nondeterministic_value(acc[c][rb]);
    }
    if (!FRESH && !(DIAG & 68) && !DIR) {
#pragma unroll
        for (int rb = 16 - LAG; rb < 16; ++rb)
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                outer[c][rb] += acc[c][rb];
                SBO_PIN_O(outer[c][rb]);
            }
    }
}

// K* pieces of one step directly (the prologue's first step)
template <int NC>
__device__ __forceinline__ void x3_kstar(const lds_char *pc, const float (&xq)[NC], const float (&yq)[NC], int g,
                                         float cexp, bool mean, KPieces<NC> &kb, double (&mu)[NC]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const f32x2v xk = lds_f2(pc + g * 32 + i * 8), yk = lds_f2(pc + 128 + g * 32 + i * 8);
        const f32x2v ak = lds_f2(pc + 256 + g * 32 + i * 8);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const float e0 = kstar1(xk.x, yk.x, xq[c], yq[c], cexp), e1 = kstar1(xk.y, yk.y, xq[c], yq[c], cexp);
            uint32_t w0, w1, w2;
            split3(e0, e1, w0, w1, w2);
            kb.h[c][i] = w0;
            kb.m[c][i] = w1;
            kb.l[c][i] = w2;
            if (mean) mu[c] += (double)fmaf(ak.x, e0, ak.y * e1);  // as in x3_half
        }
    }
}

// ---- the wide shape (variant 13): v_mfma_f32_32x32x16_bf16, four waves of
// 32 queries.  A 32x32x16 MFMA holds the SIMD's issue for 8 of its 32 cycles
// (the 16x16x32 form: 8 of 16), so the same matrix work leaves twice the
// issue slots to the K* VALU.  Lane l holds A[32 rb + (l&31)][16 s + 8(l>>5)
// + j] (A planes laid out [rb (8)][s (2)][lane][8 bf16] per half-tile, see
// pack_x3_kernel), B = K*[k = 16 s + 8(l>>5) + j][query l&31], and the 32x32
// accumulator col = l&31, rows (r&3) + 8(r>>2) + 4(l>>5).
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x16 mfma32(u32x4 a, u32x4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(a), as_bf16x8(b), c, 0, 0, 0);
}

// One half-step of one wave (wide shape): 16 sub-steps u = (rb, s), six
// MFMAs each; the next step's K* pair p = u/2 (values j = 2(p&3), +1 of
// sub-step p>>2) is evaluated at even u and split (+ mean terms, + the next
// pair's coordinates) at odd u; the finished chains of row block rb-1 are
// added into `outer` over sub-steps 2rb, 2rb+1.
template <bool FRESH, long long DIAG>
__device__ __forceinline__ void x3w_half(const lds_char *pa, const lds_char *pcn, float xq, float yq, int h,
                                         float cexp, float msc, const KPieces<2> &kb, f32x16 (&acc)[8],
                                         f32x16 (&outer)[8], KPieces<2> &nx, double &mu, uint32_t voff,
                                         const char *asrc, uint32_t adst) {
    constexpr int kStride = 4 * 1024;  // four loader waves
    const f32x16 zero = {};
    u32x4 a0 = lds_b128(pa), a1 = lds_b128(pa + kXPlane), a2 = lds_b128(pa + 2 * kXPlane);
    f32x2v xk = lds_f2(pcn + h * 32), yk = lds_f2(pcn + 128 + h * 32), ak = lds_f2(pcn + 256 + h * 32);
    f32x2v e = {0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 16; ++u) {
        const int rb = u >> 1, s = u & 1;
        u32x4 b0, b1, b2;
        if (u + 1 < 16) {
            b0 = lds_b128(pa + (u + 1) * 1024);
            b1 = lds_b128(pa + kXPlane + (u + 1) * 1024);
            b2 = lds_b128(pa + 2 * kXPlane + (u + 1) * 1024);
        }
        if (u >= 1 && u <= 12) dma16(voff, asrc + (u - 1) * kStride, adst + (u - 1) * kStride);
        const int p = u >> 1, sp = p >> 2, dp = p & 3;
        if (DIAG & 1) {
        } else if (s == 0) {
            e.x = kstar1(xk.x, yk.x, xq, yq, cexp);
            e.y = kstar1(xk.y, yk.y, xq, yq, cexp);
            SBO_PIN(e.x);
            SBO_PIN(e.y);
        } else {
            uint32_t w0, w1, w2;
            split3(e.x, e.y, w0, w1, w2);
            SBO_PIN(w0);
            SBO_PIN(w1);
            SBO_PIN(w2);
            nx.h[sp][dp] = w0;
            nx.m[sp][dp] = w1;
            nx.l[sp][dp] = w2;
            if (msc != 0.0f) {  // the next step is the mean's row block (uniform branch)
                mu += (double)fmaf(ak.x, e.x, ak.y * e.y);
                SBO_PIN(mu);
            }
            if (p < 7) {  // pair p+1: sub-step (p+1)>>2, values 2((p+1)&3), +1
                const int o = ((p + 1) >> 2) * 64 + h * 32 + ((p + 1) & 3) * 8;
                xk = lds_f2(pcn + o);
                yk = lds_f2(pcn + 128 + o);
                ak = lds_f2(pcn + 256 + o);
            }
        }
        if (!FRESH && rb > 0) {  // row block rb-1 finished a sub-step ago: half of it per sub-step
#pragma unroll
            for (int e2 = 0; e2 < 8; ++e2) {
                outer[rb - 1][8 * s + e2] += acc[rb - 1][8 * s + e2];
            }
        }
        f32x16 v = (FRESH && s == 0) ? zero : acc[rb];
        v = mfma32(a2, kb.h[s], v);
        v = mfma32(a1, kb.m[s], v);
        v = mfma32(a0, kb.l[s], v);
        v = mfma32(a1, kb.h[s], v);
        v = mfma32(a0, kb.m[s], v);
        v = mfma32(a0, kb.h[s], v);
        acc[rb] = v;
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);  // VALU
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
        }
        __builtin_amdgcn_sched_barrier(0);
        if (u + 1 < 16) {
            a0 = b0;
            a1 = b1;
            a2 = b2;
        }
    }
    if (!FRESH) outer[7] += acc[7];
}

// K* pieces of one step directly (wide shape, the prologue's first step)
__device__ __forceinline__ void x3w_kstar(const lds_char *pc, float xq, float yq, int h, float cexp, bool mean,
                                          KPieces<2> &kb, double &mu) {
#pragma unroll
    for (int sp = 0; sp < 2; ++sp)
#pragma unroll
        for (int dp = 0; dp < 4; ++dp) {
            const int o = sp * 64 + h * 32 + dp * 8;
            const f32x2v xk = lds_f2(pc + o), yk = lds_f2(pc + 128 + o), ak = lds_f2(pc + 256 + o);
            const float e0 = kstar1(xk.x, yk.x, xq, yq, cexp), e1 = kstar1(xk.y, yk.y, xq, yq, cexp);
            uint32_t w0, w1, w2;
            split3(e0, e1, w0, w1, w2);
            kb.h[sp][dp] = w0;
            kb.m[sp][dp] = w1;
            kb.l[sp][dp] = w2;
            if (mean) mu += (double)fmaf(ak.x, e0, ak.y * e1);
        }
}

// Phase stamps of the diagnostic build (DIAG & 262144), per workgroup and
// wave: cycles in [0] step top (flush, stage), [1] the half-step body,
// [2] item end, [3] vmcnt wait, [4] barrier, [5] whole half-steps, [6..8] the
// body by level, [9..11] half-steps by level.  Read by sbo_debug_x3_stamps.
constexpr int kStampFields = 16;
constexpr int kStampSlots = 1024 * 8;
__device__ unsigned long long g_x3_stamps[kStampSlots * kStampFields];

// per staged step: row block, query block, and flags
struct XStep {
    int I, qb, flags;  // bit 0: second half, bit 1: first step of its item, bit 2: last step, bit 3: valid
    int lv;            // the tile's precision level
};
constexpr int kFirst = 2, kLast = 4, kValid = 8;

// The persistent sweep.  NC = 1: eight waves (two per SIMD), wave w owns
// queries 16w .. 16w+15; NC = 2: four waves (one per SIMD), wave w owns
// queries 32w .. 32w+31.  Every wave loads an equal share of each stage.
// DIAG (timing diagnostics only, results wrong): 1 no next-step K*, 2 no A
// pieces staged, 4 no outer sums, 8 every A stage from the first tile (L2-resident);
// 16 (not a diagnostic): A pieces spread over the row blocks; 32: A fragments
// read one row block ahead instead of two; 8192 (not a diagnostic): every
// tile at the precision level its plan entry names (code << kLevelShift).
template <int NC, long long DIAG>
__global__ __launch_bounds__(NC == 1 ? 512 : 256, 1) void predict_x3_kernel(
    const char *__restrict__ ax3, const float *__restrict__ kc3, const int4 *__restrict__ desc,
    const int4 *__restrict__ rec, const int *__restrict__ seg, int P, int n_items, int nI, uint32_t a_max, int rot,
    const float *__restrict__ qx, const float *__restrict__ qy, int64_t m, int64_t ldp, float cexp, float m0,
    float *__restrict__ part, float *__restrict__ mean) {
    __shared__ __attribute__((aligned(16))) char smem[kXSmem];
    // NC = 1, 2: 16x16x32 MFMA, NC 16-query column blocks per wave; NC = 3:
    // the wide shape (32x32x16, 32 queries per wave)
    constexpr bool WIDE = NC == 3;
    constexpr int NQ = NC == 2 ? 2 : 1;                // queries per lane
    // A-stage loaders: every wave, or (DIAG & 1024, NC = 1) only waves 4-7
    constexpr bool HALF_LOAD = NC == 1 && (DIAG & 1024);
    constexpr bool LEVELS = !WIDE && (DIAG & 8192);
    constexpr int kLoaders = (NC == 1 && !HALF_LOAD) ? 8 : 4;
    constexpr int kPieces = (kXA / 1024) / kLoaders;  // A pieces per loader wave per stage (6 or 12)
    static_assert(kPieces == 6 || kPieces == 12, "the end-of-step wait below counts 6 or 12 pieces");
    const int bid = blockIdx.x;
    // (rot: diagnostic build only -- XCD b % 8 takes chunk (b + rot) % 8)
    const int rng = (P % 8 == 0) ? ((bid + rot) % 8) * (P / 8) + bid / 8 : bid;
    const int k0 = max(seg[rng], 0), k1 = min(seg[rng + 1], n_items);
    if (k0 >= k1) return;
    // DIAG & 8388608: only the workgroup's span (first to last instruction), per wave
    constexpr bool SPAN = (DIAG & 8388608) != 0;
    unsigned long long span_t0 = 0;
    if constexpr (SPAN) span_t0 = __builtin_amdgcn_s_memtime();
    const int tid = threadIdx.x, lane = tid & 63;
    const int lw = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave = loader index
    const int g = lane >> 4, r = lane & 15;
    // DIAG & 134217728 / 268435456: static issue priority 1 for waves 4-7 (the
    // second-dispatched half, which loses VALU arbitration) / for waves 0-3
    if constexpr ((DIAG & 134217728) != 0) {
        if (lw >= 4) __builtin_amdgcn_s_setprio(1);
    } else if constexpr ((DIAG & 268435456) != 0) {
        if (lw < 4) __builtin_amdgcn_s_setprio(1);
    }

    const lds_char *lds = (const lds_char *)smem;
    const int4 *rwin = reinterpret_cast<const int4 *>(smem + kXWin);
    // LDS-DMA with an SGPR base (global_load_lds_dwordx4 v_off, s_base): the
    // only per-lane operand is the byte offset lane*16
    const uint32_t voff = (uint32_t)lane * 16u;
    const uint32_t lds_smem = (uint32_t)(uintptr_t)(lds_char *)(smem);
    // (DIAG & 16777216 with HALF_LOAD: waves 0-3 load instead -- the older
    // wave of each SIMD pair, which waits at the barrier for the younger)
    const int ldr = HALF_LOAD ? ((DIAG & 16777216) ? (lw < 4 ? lw : -1) : lw - 4) : lw;  // loader index (< 0: no A pieces)
    const bool is_loader = ldr >= 0;
    const uint32_t lds_wave = lds_smem + (uint32_t)(is_loader ? ldr : 0) * 1024u;
    const uint32_t lds_rwin = lds_smem + (uint32_t)kXWin;
#define SBO_DMA16(sbase, ldst)                                                                          \
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"((const void *)(sbase)),     \
                 "{m0}"(ldst)                                                                           \
                 : "memory")
    // one half-tile stage into LDS slot `sl`: wave 0 brings the item's
    // queries (lanes 0-31 qx, 32-63 qy) and the half-tile's coordinates
    // first, then every wave its A pieces (the youngest kPieces of its
    // vector-memory operations)
#define SBO_X3_STAGE(akib_, kcf_, h_, qb_, sl_, burst_, first_)                                         \
    do {                                                                                                \
        const uint32_t d_ = lds_smem + (uint32_t)(sl_) * kXSlot;                                        \
        if (lw == 0) {                                                                                  \
            if ((first_) || WIDE) {  /* an item's queries: with its first step only */                  \
                if (lane < 32) SBO_DMA16(qx + (int64_t)(qb_) * kBN, d_ + kXA + kXC);                    \
                else SBO_DMA16(qy + (int64_t)(qb_) * kBN - 128, d_ + kXA + kXC);                        \
            }                                                                                           \
            if (lane < 32) SBO_DMA16(kc3 + (uint32_t)(kcf_) + (h_) * (kXC / 4), d_ + kXA);              \
        }                                                                                               \
        const char *s_ = a_base + ((DIAG & 8) ? 0 : (uint64_t)((akib_) + (h_) * (kXA / 1024)) * 1024u);  \
        const uint32_t w_ = lds_wave + (uint32_t)(sl_) * kXSlot;                                        \
        a_src = s_;                                                                                     \
        a_dst = w_;                                                                                     \
        if (!(DIAG & 2) && is_loader && ((burst_) || !(DIAG & 16)))                                     \
            _Pragma("unroll") for (int j = 0; j < kPieces; ++j)                                         \
                SBO_DMA16(s_ + j * kLoaders * 1024, w_ + (uint32_t)(j * kLoaders * 1024));              \
    } while (0)
    // the range's step records (plan_rec_kernel: one int4 per kept tile, in
    // sweep order) arrive in 1 KiB LDS windows of kRecWin, one window ahead
#define SBO_REC_WINDOW(w_)                                                                              \
    do {                                                                                                \
        if (lw == 1) SBO_DMA16(reinterpret_cast<const char *>(rec) + (uint64_t)(w_) * 1024u, lds_rwin + (uint32_t)((w_) & 1) * 1024u); \
    } while (0)
    auto rec_at = [&](uint32_t e) {
        const int4 d = rwin[((e / kRecWin) & 1) * kRecWin + e % kRecWin];
        return make_int4(__builtin_amdgcn_readfirstlane(d.x), __builtin_amdgcn_readfirstlane(d.y),
                         __builtin_amdgcn_readfirstlane(d.z), __builtin_amdgcn_readfirstlane(d.w));
    };
    // the range's first and one-past-last list entries
    uint32_t la_e, e_end;
    {
        const int4 da = desc[k0], db = desc[k1 - 1];
        la_e = (uint32_t)__builtin_amdgcn_readfirstlane(da.z);
        e_end = (uint32_t)__builtin_amdgcn_readfirstlane(db.z) + (uint32_t)(__builtin_amdgcn_readfirstlane(db.w) & 0xffff);
    }
    SBO_REC_WINDOW(la_e / kRecWin);
    SBO_REC_WINDOW(la_e / kRecWin + 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int la_h = 0;

    // this wave's share of every A stage starts at a_base (+ the stage's offset)
    const char *a_base = ax3 + (is_loader ? ldr : 0) * 1024;
    const char *a_src = ax3;  // this wave's A pieces of the last staged step (spread mode)
    uint32_t a_dst = 0;
    // the record of entry la_e, read when la_e became current (one stage call
    // ahead of its use: the LDS latency off the step top)
    int4 r_cur = rec_at(la_e);
    auto stage = [&](int sl, bool burst) {
        const int4 r = r_cur;
        XStep s;
        s.I = min(r.w & 0xffff, nI - 1);
        s.qb = r.z;
        s.flags = la_h | ((r.w & kRecFirst) && la_h == 0 ? kFirst : 0) | ((r.w & kRecLast) && la_h == 1 ? kLast : 0) |
                  kValid;
        s.lv = LEVELS ? min((r.w >> 16) & 3, 2) : 0;
        SBO_X3_STAGE(min((uint32_t)r.x, a_max), r.y, la_h, r.z, sl, burst, (s.flags & kFirst) != 0);
        la_h ^= 1;
        if (la_h == 0) {
            ++la_e;
            // window w + 1 goes into the buffer of window w - 1 once entry
            // 64 w + 1 is current: every wave read that buffer's last entry
            // (64 w - 1) at least one barrier ago (at 64 w the slower waves
            // may still be reading it in this same step)
            if (la_e % kRecWin == 1) SBO_REC_WINDOW(la_e / kRecWin + 1);
            if (la_e < e_end) r_cur = rec_at(la_e);
        }
        return s;
    };

    XStep s0 = stage(0, true), s1 = {0, 0, 0, 0}, s2 = {0, 0, 0, 0};
    if (la_e < e_end) s1 = stage(1, true);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    // the lane's queries in the block: qo + 16 c (c < NQ)
    const int qo = WIDE ? lw * 32 + (lane & 31) : lw * 16 * NC + r;
    constexpr int kCB = NC == 2 ? 2 : 1, kRB = WIDE ? 8 : 16;
    typedef std::conditional_t<WIDE, f32x16, f32x4> AccT;
    AccT acc[kCB][kRB], outer[kCB][kRB];
#pragma unroll
    for (int c = 0; c < kCB; ++c)
#pragma unroll
        for (int rb = 0; rb < kRB; ++rb) {
            acc[c][rb] = AccT{};
            outer[c][rb] = acc[c][rb];
        }
    double mu[NQ];
    KPieces<WIDE ? 2 : NC> kb, nx;
    // the lane's query coordinates of the item whose K* is being built: read
    // from the slot of an item's first step only (its stage alone carries them)
    float xq[NQ], yq[NQ];
    {
        const lds_char *pq = lds + kXA + kXC;
#pragma unroll
        for (int c = 0; c < NQ; ++c) {
            mu[c] = 0.0;
            xq[c] = lds_f(pq + (qo + 16 * c) * 4);
            yq[c] = lds_f(pq + (kBN + qo + 16 * c) * 4);
        }
        if constexpr (WIDE)
            x3w_kstar(lds + kXA, xq[0], yq[0], lane >> 5, cexp, s0.I == nI - 1, kb, mu[0]);
        else
            x3_kstar<NC>(lds + kXA, xq, yq, g, cexp, s0.I == nI - 1, kb, mu);
    }
    // deferred outputs of the item finished in the previous step (stored at
    // the top of the next step, before its stage DMA, so that the vmcnt count
    // at the end of every step is the A pieces of one stage)
    bool pend = false, pend_mean = false;
    float pend_s[NQ], pend_mu[NQ];
    int64_t pend_q = 0;
    int pend_I = 0;
    auto flush = [&]() {
        if (pend && lane < (WIDE ? 32 : 16)) {
#pragma unroll
            for (int c = 0; c < NQ; ++c) {
                const int64_t q = pend_q + 16 * c;
                if (q < m) {
                    part[(int64_t)pend_I * ldp + q] = pend_s[c];
                    if (pend_mean) mean[q] = pend_mu[c];
                }
            }
        }
        pend = false;
    };
    int cur = 0;
    bool more = true;
    constexpr bool STAMP = (DIAG & 262144) != 0;
    unsigned long long stc[12] = {};
#define SBO_STAMP(t_)                                                                          \
    do {                                                                                       \
        __builtin_amdgcn_sched_barrier(0);                                                     \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");           \
        __builtin_amdgcn_sched_barrier(0);                                                     \
    } while (0)
    // one half-step; items are whole tiles, so the steps alternate FRESH
    // (first half: chains from zero) and second halves (which may end an item)
    auto half_step = [&](auto fresh_tag) {
        constexpr bool FRESH = decltype(fresh_tag)::value;
        unsigned long long t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0, t5 = 0;
        if constexpr (STAMP) SBO_STAMP(t0);
        if (FRESH) flush();
        const bool issue = la_e < e_end;
        const int nslot = cur == 0 ? 2 : cur - 1;  // (cur + 2) % 3
        s2 = issue ? stage(nslot, false) : XStep{0, 0, 0, 0};
        // A pieces the staged tile's level needs (plane p = pieces p*kPieces/3 ..)
        const int np2 = LEVELS ? (kPieces / 3) * (3 - s2.lv) : kPieces;
        if (!issue) a_dst = lds_wave + (uint32_t)nslot * kXSlot;  // spread mode: a harmless re-stage into the free slot
        const int cslot = cur == 2 ? 0 : cur + 1;  // (cur + 1) % 3: the next step's coordinates
        const lds_char *pa = lds + cur * kXSlot + lane * 16;
        const lds_char *pcn = lds + cslot * kXSlot + kXA;
        const lds_char *pqn = pcn + kXC;
        const bool nvalid = (s1.flags & kValid) != 0;
        const float msc = nvalid && s1.I == nI - 1 ? 1.0f : 0.0f;
        if (!FRESH) {
            // this step may end its item: the item's mean terms are all in
            // (its K* were built one step ahead); close it before the next
            // item's terms start
            if ((s0.flags & kLast) && s0.I == nI - 1) {
#pragma unroll
                for (int c = 0; c < NQ; ++c) {
                    double u = mu[c];
                    if (!WIDE) u += __shfl_xor(u, 16);
                    u += __shfl_xor(u, 32);
                    pend_mu[c] = (float)((double)m0 + u);
                }
            }
            if (nvalid && (s1.flags & kFirst))
#pragma unroll
                for (int c = 0; c < NQ; ++c) mu[c] = 0.0;
        }
        if (WIDE || (nvalid && (s1.flags & kFirst))) {
#pragma unroll
            for (int c = 0; c < NQ; ++c) {
                xq[c] = lds_f(pqn + (qo + 16 * c) * 4);
                yq[c] = lds_f(pqn + (kBN + qo + 16 * c) * 4);
            }
        }
        if constexpr (STAMP) SBO_STAMP(t1);
        if constexpr (WIDE)
            x3w_half<FRESH, DIAG>(pa, pcn, xq[0], yq[0], lane >> 5, cexp, msc, kb, acc[0], outer[0], nx, mu[0],
                                  voff, a_src, a_dst);
        else {
            // the body by the tile's level, the next step's, and whether the
            // next step is the mean's row block (all uniform: one branch here,
            // none inside the body's MFMA region)
            // (DIAG & 2^31: the one-product bodies by the mean test, at compile time)
            constexpr bool MSPLIT = (DIAG & 2147483648LL) != 0;
            if (LEVELS && s0.lv == 2 && (DIAG & 1073741824) && nvalid && s1.lv == 2) {
                if (MSPLIT && msc == 0.0f)
                    x3_half<NC, FRESH, DIAG, kPieces, 2, true, 0>(pa, pcn, xq, yq, g, cexp, msc, kb, acc, outer, nx,
                                                                  mu, voff, a_src, a_dst, is_loader, np2);
                else
                    x3_half<NC, FRESH, DIAG, kPieces, 2, true, MSPLIT ? 1 : -1>(pa, pcn, xq, yq, g, cexp, msc, kb, acc,
                                                                               outer, nx, mu, voff, a_src, a_dst,
                                                                               is_loader, np2);
            } else if (LEVELS && s0.lv == 2) {
                if (MSPLIT && msc == 0.0f)
                    x3_half<NC, FRESH, DIAG, kPieces, 2, false, 0>(pa, pcn, xq, yq, g, cexp, msc, kb, acc, outer, nx,
                                                                   mu, voff, a_src, a_dst, is_loader, np2);
                else
                    x3_half<NC, FRESH, DIAG, kPieces, 2, false, MSPLIT ? 1 : -1>(pa, pcn, xq, yq, g, cexp, msc, kb,
                                                                                acc, outer, nx, mu, voff, a_src,
                                                                                a_dst, is_loader, np2);
            } else if (LEVELS && s0.lv == 1 && (DIAG & 1073741824) && (DIAG & 524288) && nvalid && s1.lv == 2)
                x3_half<NC, FRESH, DIAG, kPieces, 1, true>(pa, pcn, xq, yq, g, cexp, msc, kb, acc, outer, nx, mu, voff,
                                                           a_src, a_dst, is_loader, np2);
            else if (LEVELS && s0.lv == 1)
                x3_half<NC, FRESH, DIAG, kPieces, 1>(pa, pcn, xq, yq, g, cexp, msc, kb, acc, outer, nx, mu, voff,
                                                     a_src, a_dst, is_loader, np2);
            else
                x3_half<NC, FRESH, DIAG, kPieces>(pa, pcn, xq, yq, g, cexp, msc, kb, acc, outer, nx, mu, voff, a_src,
                                                  a_dst, is_loader, np2);
        }
        if constexpr (STAMP) SBO_STAMP(t2);
        if (!FRESH && (s0.flags & kLast)) {
            // item done: column sums of V^2 over its rows (lanes l, l+16, l+32,
            // l+48 hold four row quarters of column l&15 of every block)
            if (DIAG & 64) {
#pragma unroll
                for (int c = 0; c < kCB; ++c)
#pragma unroll
                    for (int rb = 0; rb < kRB; ++rb) {
                        outer[c][rb] = acc[c][rb];
                        acc[c][rb] = AccT{};
                    }
            }
            pend = true;
            pend_I = s0.I;
            pend_q = (int64_t)s0.qb * kBN + qo;
            pend_mean = s0.I == nI - 1;
            constexpr int kE = WIDE ? 16 : 4;
#pragma unroll
            for (int c = 0; c < kCB; ++c) {
                // four independent f64 chains (element e of every block), then
                // combined: the 64-term sum off one dependent fma chain
                double sq[kE > 4 ? 4 : kE] = {};
#pragma unroll
                for (int rb = 0; rb < kRB; ++rb)
#pragma unroll
                    for (int e = 0; e < kE; ++e) {
                        sq[e & 3] = fma((double)outer[c][rb][e], (double)outer[c][rb][e], sq[e & 3]);
                        outer[c][rb][e] = 0.0f;
                    }
                double sv = (sq[0] + sq[1]) + (sq[2] + sq[3]);
                if (!WIDE) sv += __shfl_xor(sv, 16);
                sv += __shfl_xor(sv, 32);
                pend_s[c] = (float)sv;
            }
        }
        if constexpr (STAMP) SBO_STAMP(t3);
        // retire stage i+1: its queries and coordinates (wave 0) precede its
        // A pieces and were retired one step earlier; leave stage i+2's A in flight
        if ((issue || (DIAG & 16)) && !(DIAG & 2) && is_loader) {
            if constexpr (kPieces == 12) {
                asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
            } else if constexpr (LEVELS && (DIAG & 16384)) {  // stage i+2 issued np2 pieces
                if (np2 == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
                else if (np2 == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
            }
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if constexpr (STAMP) SBO_STAMP(t4);
        if constexpr (DIAG & 512)  // timing only: no step barrier (races on the slots)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        else
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if constexpr (STAMP) {
            SBO_STAMP(t5);
            const int lvs = LEVELS ? s0.lv : 0;
            stc[0] += t1 - t0;
            stc[1] += t2 - t1;
            stc[2] += t3 - t2;
            stc[3] += t4 - t3;
            stc[4] += t5 - t4;
            stc[5] += t5 - t0;
            stc[6 + lvs] += t2 - t1;
            stc[9 + lvs] += 1;
        }
        more = nvalid;
        s0 = s1;
        s1 = s2;
        kb = nx;
        cur = cslot;
    };
    do {
        half_step(std::integral_constant<bool, true>{});
        half_step(std::integral_constant<bool, false>{});
    } while (more);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may land after the workgroup ends
    flush();
    if constexpr (SPAN) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        const int slot = bid * 8 + lw;
        if (lane == 0 && slot < kStampSlots) {
            g_x3_stamps[(size_t)slot * kStampFields + 5] = t1 - span_t0;
            g_x3_stamps[(size_t)slot * kStampFields + 9] = 1;
        }
    }
    if constexpr (STAMP) {
        const int slot = bid * 8 + lw;
        if (lane == 0 && slot < kStampSlots)
#pragma unroll
            for (int j = 0; j < 12; ++j) g_x3_stamps[(size_t)slot * kStampFields + j] = stc[j];
    }
#undef SBO_STAMP
#undef SBO_X3_STAGE
#undef SBO_REC_WINDOW
#undef SBO_DMA16
}

// Split the f32 packed operand (tiles T0 .. T1-1, tile_offset layout) into
// the three bf16 planes of the x3 layout: tile T, half h, plane p, row block
// rb, lane l = 16 g + r holds A[16 rb + r][32 h + 8 g + j], j = 0..7, at
// byte T*2*kXA + h*kXA + p*kXPlane + rb*1024 + l*16 + 2j.
// wide = 1: the 32x32x16 layout of the wide shape, lane l of 1 KiB run
// u = 2 rb + s holds A[32 rb + (l&31)][32 h + 16 s + 8(l>>5) + j].
__global__ __launch_bounds__(256) void pack_x3_kernel(const float *__restrict__ aug, int64_t T0, int64_t nt,
                                                      int wide, char *__restrict__ ax3) {
    const int64_t id = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (id >= nt * 2048) return;
    const int lane = (int)(id & 63), rb = (int)((id >> 6) & 15), h = (int)((id >> 10) & 1);
    const int64_t T = T0 + (id >> 11);
    const int row = wide ? (rb >> 1) * 32 + (lane & 31) : rb * 16 + (lane & 15);
    const int k0 = wide ? kXH * h + 16 * (rb & 1) + 8 * (lane >> 5) : kXH * h + 8 * (lane >> 4);
    const float *src = aug + T * kTileFloats;
    u32x4 w0, w1, w2;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const int k = k0 + 2 * d;
        uint32_t a, b, c;
        split3(src[tile_offset(k, row)], src[tile_offset(k + 1, row)], a, b, c);
        w0[d] = a;
        w1[d] = b;
        w2[d] = c;
    }
    char *dst = ax3 + T * (2 * kXA) + h * kXA + rb * 1024 + lane * 16;
    *reinterpret_cast<u32x4 *>(dst) = w0;
    *reinterpret_cast<u32x4 *>(dst + kXPlane) = w1;
    *reinterpret_cast<u32x4 *>(dst + 2 * kXPlane) = w2;
}

// Per k-tile coordinates in natural order per half: kc3[t*256 + h*128 + c*32 + i]
// = (x, y, sf2 alpha, 0)[c] of k = 64t + 32h + i, from the kcoord layout
// (k = 4p + g of a tile at g*16 + p).
__global__ void pack_kc3_kernel(const float *__restrict__ kcoord, int64_t nkt, float *__restrict__ kc3) {
    const int64_t id = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (id >= nkt * 256) return;
    const int64_t t = id >> 8;
    const int o = (int)(id & 255), h = o >> 7, c = (o >> 5) & 3, i = o & 31;
    const int kk = kXH * h + i;
    kc3[id] = c < 3 ? kcoord[t * (3 * kBK) + c * kBK + (kk & 3) * 16 + (kk >> 2)] : 0.0f;
}

}  // namespace

size_t x3_operand_bytes(int64_t npad) { return (size_t)total_tiles(npad / kBM) * 2 * kXA; }
size_t x3_coord_bytes(int64_t npad) { return (size_t)(npad / kBK) * 256 * sizeof(float); }

hipError_t launch_pack_x3(hipStream_t s, const float *aug, const float *kcoord, int64_t npad, int64_t I0, int wide,
                          char *ax3, float *kc3) {
    const int64_t nI = npad / kBM;
    const int64_t T0 = tile_start(I0), T1 = tile_start(nI);
    if (ax3 && T1 > T0) {
        const int64_t th = (T1 - T0) * 2048;
        hipLaunchKernelGGL(pack_x3_kernel, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, s, aug, T0, T1 - T0, wide,
                           ax3);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (!kc3) return hipSuccess;
    const int64_t nkt = npad / kBK;
    hipLaunchKernelGGL(pack_kc3_kernel, dim3((unsigned)((nkt * 256 + 255) / 256)), dim3(256), 0, s, kcoord, nkt, kc3);
    return hipGetLastError();
}

hipError_t read_x3_stamps(double *out, int n) {
    std::vector<unsigned long long> h((size_t)kStampSlots * kStampFields);
    hipError_t e = hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_x3_stamps), h.size() * sizeof(unsigned long long));
    if (e != hipSuccess) return e;
    for (int j = 0; j < n; ++j) out[j] = 0.0;
    // out[0..11]: summed over all waves; out[12 + 12 w + j]: over wave index w
    // of every workgroup; out[108 + b]: workgroup b's loop cycles (mean over its waves)
    for (size_t sl = 0; sl < (size_t)kStampSlots; ++sl) {
        for (int j = 0; j < 12; ++j) {
            const double v = (double)h[sl * kStampFields + j];
            if (j < n) out[j] += v;
            const int o = 12 + 12 * (int)(sl % 8) + j;
            if (o < n) out[o] += v;
        }
        const int o = 108 + (int)(sl / 8);
        if (o < n) out[o] += (double)h[sl * kStampFields + 5] / 8.0;
    }
    std::fill(h.begin(), h.end(), 0ull);  // reset for the next read
    return hipMemcpyToSymbol(HIP_SYMBOL(g_x3_stamps), h.data(), h.size() * sizeof(unsigned long long));
}

hipError_t launch_predict_x3(hipStream_t s, const char *ax3, const float *kc3, const int4 *desc, const int4 *rec,
                             const int *seg, int P, int n_items, int nI, const float *qx, const float *qy, int64_t m,
                             int64_t ldp, float cexp, float m0, float *part, float *mean, int variant) {
    // the largest tile offset a record may name (KiB): keeps every staged address inside ax3
    const int64_t amax = (total_tiles(nI) - 1) * (2 * kXA / 1024);
    if (nI <= 0 || amax > 0xffffffffll) return hipErrorInvalidValue;
    const uint32_t a_max = (uint32_t)amax;
    int rot = 0;
#ifdef SBO_DIAG
    if (const char *e = getenv("SBO_XCD_ROT")) rot = std::clamp(atoi(e), 0, 7);
#endif
#define SBO_X3_LAUNCH(NC, D) \
    hipLaunchKernelGGL((predict_x3_kernel<NC, D>), dim3((unsigned)P), dim3(NC == 1 ? 512 : 256), 0, s, ax3, kc3, desc, rec, \
                       seg, P, n_items, nI, a_max, rot, qx, qy, m, ldp, cexp, m0, part, mean)
    switch (variant) {
        case 2: SBO_X3_LAUNCH(2, 16); break;   // four waves of 32 queries
        case 9: SBO_X3_LAUNCH(1, 0); break;    // A pieces in a burst at the top of the step
        case 10: SBO_X3_LAUNCH(1, 48); break;  // A fragments one row block ahead
        case 13: SBO_X3_LAUNCH(3, 16); break;  // wide shape: 32x32x16 MFMA, four waves of 32 queries
        case 22: SBO_X3_LAUNCH(1, 16); break;    // variant 3 with every tile at full precision
#ifdef SBO_DIAG
        case 4: SBO_X3_LAUNCH(2, 17); break;   // diagnostics: no next-step K*
        case 5: SBO_X3_LAUNCH(2, 18); break;   //   no A pieces
        case 6: SBO_X3_LAUNCH(1, 17); break;   //   no next-step K*
        case 7: SBO_X3_LAUNCH(1, 18); break;   //   no A pieces
        case 8: SBO_X3_LAUNCH(1, 24); break;   //   every stage from the first tile
        case 11: SBO_X3_LAUNCH(1, 80); break;  // diagnostics: one chain per item, no outer sums
        case 12: SBO_X3_LAUNCH(1, 81); break;  //   and no next-step K*
        case 14: SBO_X3_LAUNCH(3, 17); break;  //   diagnostics: no next-step K*
        case 15: SBO_X3_LAUNCH(1, 144); break;  // schedule A/B: four VALU per MFMA gap
        case 16: SBO_X3_LAUNCH(1, 272); break;  //   the compiler's own interleave
        case 17: SBO_X3_LAUNCH(1, 528); break;  // diagnostics: no step barrier (wrong results)
        case 18: SBO_X3_LAUNCH(1, 529); break;  //   and no next-step K*
        case 19: SBO_X3_LAUNCH(1, 1040); break;  // A stage loaded by waves 4-7 only (12 pieces each)
        case 20: SBO_X3_LAUNCH(1, 2064); break;  // diagnostics: 3 of the 6 split products
        case 21: SBO_X3_LAUNCH(1, 4112); break;  //   1 of the 6
        case 23: SBO_X3_LAUNCH(1, 8208); break;  // variant 3 with A fragments two row blocks ahead
        case 24: SBO_X3_LAUNCH(1, 24624); break;  // variant 3 issuing only the A pieces a level reads
        case 25: SBO_X3_LAUNCH(1, 4113); break;   // diagnostics: 1 product, no next-step K*
        case 26: SBO_X3_LAUNCH(1, 4114); break;   //   1 product, no A pieces
        case 27: SBO_X3_LAUNCH(1, 4115); break;   //   1 product, neither
        case 28: SBO_X3_LAUNCH(1, 4116); break;   //   1 product, no outer sums
        case 29: SBO_X3_LAUNCH(1, 4119); break;   //   1 product, none of the three
        case 30: SBO_X3_LAUNCH(1, 41008); break;  // variant 3 with the outer sums two blocks behind at every level
        case 31: SBO_X3_LAUNCH(1, 36880); break;  // diagnostics: 1 product, outer sums two blocks behind
        case 32: SBO_X3_LAUNCH(1, 8240); break;   // variant 3 with A fragments one block ahead at every level
        case 33: SBO_X3_LAUNCH(1, 139312); break;  // variant 3 with A fragments 8 / 3 blocks ahead at one / three products
        case 34: SBO_X3_LAUNCH(1, 69648); break;  // diagnostics (A 4 ahead): 1 product
        case 35: SBO_X3_LAUNCH(1, 70160); break;  //   1 product, no step barrier (wrong results)
        case 36: SBO_X3_LAUNCH(1, 69651); break;  //   1 product, no next-step K*, no A pieces
        case 37: SBO_X3_LAUNCH(1, 70163); break;  //   and no barrier
        case 38: SBO_X3_LAUNCH(1, 69655); break;  //   no K*, no A pieces, no outer sums
        case 39: SBO_X3_LAUNCH(1, 335920 + 33554432 + 1073741824 + 67108864); break;  // variant 3 with phase stamps (sbo_debug_x3_stamps)
        case 41: SBO_X3_LAUNCH(1, 1122352); break;  // diagnostics: variant 3 with the K* split reduced to kh
        // A/B (correct results, measured no faster: DESIGN.md section 10):
        case 42: SBO_X3_LAUNCH(1, 73776 + 2097152); break;  // variant 3, one-product tiles straight into the outer sums
        case 43: SBO_X3_LAUNCH(1, 73776 + 6291456); break;  //   and three-product tiles too
        case 46: SBO_X3_LAUNCH(1, 73776 + 33554432 + 1073741824 + 67108864 + 8388608); break;  // variant 3 recording only each workgroup's span
        case 47: SBO_X3_LAUNCH(1, 73776 + 1024 + 16777216); break;  // variant 3, A stage loaded by waves 0-3 only
        case 48: SBO_X3_LAUNCH(1, 73776 + 1024); break;     // variant 3, A stage loaded by waves 4-7 only
        case 49: SBO_X3_LAUNCH(1, 73776); break;  // variant 3 with the next K* coordinates read at ph 3 (round-2 default)
        case 51: SBO_X3_LAUNCH(1, 73776 + 33554432 + 134217728); break;  // variant 3, waves 4-7 at issue priority 1
        case 52: SBO_X3_LAUNCH(1, 73776 + 33554432 + 268435456); break;  // variant 3, waves 0-3 at issue priority 1
        case 53: SBO_X3_LAUNCH(1, 73776 + 33554432 + 536870912); break;  // diagnostics: variant 3 with a one-multiply K*
        case 54: SBO_X3_LAUNCH(1, 73776 + 33554432 + 536870912 + 1048576); break;  //   and the split reduced to kh
        case 55: SBO_X3_LAUNCH(1, 73776 + 33554432); break;  // variant 3 without the kh-only split (the default before it)
        case 56: SBO_X3_LAUNCH(1, 73776 + 33554432 + 1073741824 + 524288); break;  // variant 3, kh-only split from three-product steps too (slower)
        case 57: SBO_X3_LAUNCH(1, 73776 + 33554432 + 1073741824); break;  // variant 3 reading sf2 alpha before every step (the default before)
        case 60: SBO_X3_LAUNCH(2, 73776 + 33554432 + 1073741824 + 67108864); break;  // variant 3's options, four waves of 32 queries (one per SIMD)
        case 61: SBO_X3_LAUNCH(2, 73776 + 33554432 + 67108864); break;  //   without the kh-only split bodies
        case 59: SBO_X3_LAUNCH(1, 73776 + 33554432 + 1073741824 + 4294967296LL); break;  // variant 3, mean terms by a select (no branch)
        case 58: SBO_X3_LAUNCH(1, 73776 + 33554432 + 1073741824 + 67108864 + 2147483648LL); break;  // variant 3, one-product bodies split by the mean test at compile time
#endif
        default: SBO_X3_LAUNCH(1, 73776 + 33554432 + 1073741824 + 67108864); break;  // 3: eight waves of 16 queries, A pieces spread, tile levels, A 1 / 2 / 4 blocks ahead, next coordinates at ph 1, kh-only split between one-product steps, sf2 alpha read only before the mean's row block
    }
#undef SBO_X3_LAUNCH
    return hipGetLastError();
}

}  // namespace sbo
