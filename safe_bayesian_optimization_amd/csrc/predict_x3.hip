// predict_x3.hip -- the predictive sweep (a3+a4) on bf16 MFMA with split
// operands: f32-accurate V = A K*^T at 6/16 of the f32 MFMA cycles.
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
// and is added into an f32 outer sum once the tile is done.  Every tile runs
// at the precision level its plan entry names (six, three or one product(s)).
//
// Staging: three LDS slots, stage i+2 issued during step i by LDS-DMA
// (global_load_lds_dwordx4 from inline asm: the query and coordinate pieces
// at the top of the step, the A pieces one per row block between the MFMAs),
// retired by a counted vmcnt at the end of step i+1; the slot also carries
// the half-tile's coordinates, sf2 alpha and the item's 128 query
// coordinates, so the K* of step i+1 is computed during step i, beside its
// MFMAs.
//
// This is the product build's one code path (SBO_OPT_KERNEL_VARIANT 3, and 22
// = the same kernel over a plan without precision levels).  Every A/B and
// timing variant of rounds 1-3 (the DIAG template mask: other shapes, stage
// burst, phase stamps, work left out) lives in diag/predict_x3_diag.hip, built
// only into lib/libsbo_diag.so; its variant 3 is this kernel.
#include <cstdint>
#include <vector>

#include "sbo_internal.hpp"

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
constexpr int kXWin = kXSlots * kXSlot;  // the step-record windows follow the slots
constexpr int kXSmem = kXWin + 4096;
constexpr int kRecWin = 64;              // step records (int4) per 1 KiB LDS window
constexpr int kLoaders = 8;              // every wave loads an eighth of each A stage
constexpr int kPieces = (kXA / 1024) / kLoaders;  // 6 A pieces per wave per stage (2 per plane)
constexpr int kStride = kLoaders * 1024;          // a wave's consecutive pieces
static_assert(kPieces == 6, "the end-of-step wait below counts 6 pieces");

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
typedef float f32x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2v lds_f2(const lds_char *p) {
    return *reinterpret_cast<const __attribute__((address_space(3))) f32x2v *>(p);
}

// One LDS-DMA piece under a wave-uniform EXEC mask (0: no lane moves data,
// but the instruction still issues and counts in vmcnt, so the step's wait
// count stays static) -- no control flow in the scheduled MFMA region.
// s_nop: the M0 write -> LDS-DMA hazard.
__device__ __forceinline__ void dma16_masked(uint32_t voff, const void *sbase, uint32_t ldst, uint64_t mask) {
    uint64_t sv;
    asm volatile("s_mov_b64 %0, exec\n\ts_and_b64 exec, exec, %4\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\t"
                 "s_mov_b64 exec, %0"
                 : "=&s"(sv)
                 : "v"(voff), "s"(sbase), "{m0}"(ldst), "s"(mask)
                 : "memory", "scc");
}

// K* pieces of a step (lane (g, r): k = 8g + j of the half-tile, query 16 w + r)
struct KPieces {
    u32x4 h, m, l;
};

__device__ __forceinline__ float kstar1(float xk, float yk, float xq, float yq, float cexp) {
    const float dx = xk - xq, dy = yk - yq;
    return fast_exp2(fmaf(dy, dy, dx * dx) * cexp);
}

// Pin a value's computation to this point of the instruction stream (the
// IR-level sinking passes ignore sched_barrier and would otherwise bunch the
// next step's K* work after the last MFMA), in an arch VGPR.
#define SBO_PIN(v) asm volatile("" : "+v"(v))

// One half-step of one wave: 16 row blocks x 6, 3 or 1 MFMA(s) (the tile's
// precision level LV) on this slot's A planes and this step's K* pieces kb,
// with the next step's K* pieces and its mean terms (scaled by msc: 1 for the
// last row block, else 0) built beside them: pair i of the lane's eight k in
// row blocks 4i .. 4i+3 (evaluate at rb = 4i, 4i+1, split at 4i+2, mean terms
// at 4i+3; the next pair's coordinates are read at 4i+1).
//   FRESH: first half of a tile (the chains start from zero); otherwise the
//   finished chains of each row block are added into `outer` LAG blocks later
//   (2 / 4 / 8 at six / three / one product(s): off the MFMA's result latency).
//   LV: 0 all six products, 1 the three largest (a1 kh + a0 km + a0 kh), 2 a0
//   kh alone; the A planes a level leaves out are not read from LDS, and A
//   fragments are read AH = 1 / 2 / 4 blocks ahead so the LDS latency stays
//   covered however few MFMAs a block has.
//   KHN: the next step runs at one product too: its K* pieces are kh alone,
//   the split skipped (a one-product step reads no other piece, so the
//   results are bitwise those of the full split).
// The stage two steps ahead (asrc -> adst) is issued here: this wave's A
// piece j between row blocks j and j + 1 -- planes the staged tile's level
// does not read under an all-zero EXEC mask (npieces: the pieces it reads).
template <bool FRESH, int LV, bool KHN>
__device__ __forceinline__ void x3_half(const lds_char *pa, const lds_char *pcn, float xq, float yq, int g,
                                        float cexp, float msc, const KPieces &kb, f32x4 (&acc)[16],
                                        f32x4 (&outer)[16], KPieces &nx, double &mu, uint32_t voff, const char *asrc,
                                        uint32_t adst, int npieces) {
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
    constexpr bool P1 = LV <= 1, P2 = LV == 0;  // planes a1, a2 in use
    constexpr int NPROD = LV == 0 ? 6 : (LV == 1 ? 3 : 1);
    constexpr int LAG = LV == 0 ? 2 : (LV == 1 ? 4 : 8);
    constexpr int AH = LV == 2 ? 4 : (LV == 1 ? 2 : 1);
    u32x4 f0[16], f1[16], f2[16];
#pragma unroll
    for (int r = 0; r < AH; ++r) {
        f0[r] = lds_b128(pa + r * 1024);
        if constexpr (P1) f1[r] = lds_b128(pa + kXPlane + r * 1024);
        if constexpr (P2) f2[r] = lds_b128(pa + 2 * kXPlane + r * 1024);
    }
    // coordinates of pair 0 (sf2 alpha only before the mean's row block)
    f32x2v xk = lds_f2(pcn + g * 32), yk = lds_f2(pcn + 128 + g * 32), ak = {0.f, 0.f};
    if (msc != 0.0f) ak = lds_f2(pcn + 256 + g * 32);
    f32x2v e;
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
        // ---- the next step's K*, pair i over row blocks 4i .. 4i+3
        const int i = rb >> 2, ph = rb & 3;
        if (ph <= 1) {
            float ev = kstar1(ph == 0 ? xk.x : xk.y, ph == 0 ? yk.x : yk.y, xq, yq, cexp);
            SBO_PIN(ev);
            if (ph == 0) e.x = ev; else e.y = ev;
            if (ph == 1 && i < 3) {  // the next pair's x, y
                xk = lds_f2(pcn + g * 32 + (i + 1) * 8);
                yk = lds_f2(pcn + 128 + g * 32 + (i + 1) * 8);
            }
        } else if (ph == 2) {
            if constexpr (KHN) {  // the next step runs at one product: kh alone
                uint32_t w0 = pk_bf16(e.x, e.y);
                SBO_PIN(w0);
                nx.h[i] = w0;
            } else {
                uint32_t w0, w1, w2;
                split3(e.x, e.y, w0, w1, w2);
                SBO_PIN(w0);
                SBO_PIN(w1);
                SBO_PIN(w2);
                nx.h[i] = w0;
                nx.m[i] = w1;
                nx.l[i] = w2;
            }
        } else {
            if (msc != 0.0f) {  // the next step is the mean's row block
                // the pair's terms in f32 (one rounding of a two-term sum,
                // the order of K*'s own), accumulated in f64
                mu += (double)fmaf(ak.x, e.x, ak.y * e.y);
                SBO_PIN(mu);
            }
            if (i < 3 && msc != 0.0f) ak = lds_f2(pcn + 256 + g * 32 + (i + 1) * 8);
        }
        if (rb >= 1 && rb <= kPieces) {
            const uint32_t mh = (uint32_t)__builtin_amdgcn_readfirstlane(rb <= npieces ? -1 : 0);
            dma16_masked(voff, asrc + (rb - 1) * kStride, adst + (rb - 1) * kStride, ((uint64_t)mh << 32) | mh);
        }
        // the finished chains of block rb - LAG
        if (!FRESH && rb >= LAG) outer[rb - LAG] += acc[rb - LAG];
        f32x4 v = FRESH ? zero : acc[rb];
        if constexpr (P2) {
            v = mfma(a2, kb.h, v);
            v = mfma(a1, kb.m, v);
            v = mfma(a0, kb.l, v);
        }
        if constexpr (P1) {
            v = mfma(a1, kb.h, v);
            v = mfma(a0, kb.m, v);
        }
        v = mfma(a0, kb.h, v);
        acc[rb] = v;
        // interleave: each MFMA followed by two VALU and one LDS read, so the
        // vector work issues in the matrix pipe's shadow (a bf16 MFMA holds
        // the SIMD's issue for 8 of its 16 cycles)
#pragma unroll
        for (int j = 0; j < NPROD; ++j) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // VALU
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    if (!FRESH) {
#pragma unroll
        for (int rb = 16 - LAG; rb < 16; ++rb) outer[rb] += acc[rb];
    }
}

// K* pieces of one step directly (the prologue's first step)
__device__ __forceinline__ void x3_kstar(const lds_char *pc, float xq, float yq, int g, float cexp, bool mean,
                                         KPieces &kb, double &mu) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const f32x2v xk = lds_f2(pc + g * 32 + i * 8), yk = lds_f2(pc + 128 + g * 32 + i * 8);
        const f32x2v ak = lds_f2(pc + 256 + g * 32 + i * 8);
        const float e0 = kstar1(xk.x, yk.x, xq, yq, cexp), e1 = kstar1(xk.y, yk.y, xq, yq, cexp);
        uint32_t w0, w1, w2;
        split3(e0, e1, w0, w1, w2);
        kb.h[i] = w0;
        kb.m[i] = w1;
        kb.l[i] = w2;
        if (mean) mu += (double)fmaf(ak.x, e0, ak.y * e1);  // as in x3_half
    }
}

// per staged step: row block, query block, flags and the tile's precision level
struct XStep {
    int I, qb, flags;  // bit 0: second half, bit 1: first step of its item, bit 2: last step, bit 3: valid
    int lv;
};
constexpr int kFirst = 2, kLast = 4, kValid = 8;

// The persistent sweep: eight waves (two per SIMD), wave w owns queries
// 16w .. 16w+15; every wave loads an eighth of each stage's A planes.
__global__ __launch_bounds__(512, 1) void predict_x3_kernel(
    const char *__restrict__ ax3, const float *__restrict__ kc3, const int4 *__restrict__ desc,
    const int4 *__restrict__ rec, const int *__restrict__ seg, int P, int n_items, int nI, uint32_t a_max,
    const float *__restrict__ qx, const float *__restrict__ qy, int64_t m, int64_t ldp, float cexp, float m0,
    float *__restrict__ part, float *__restrict__ mean) {
    __shared__ __attribute__((aligned(16))) char smem[kXSmem];
    const int bid = blockIdx.x;
    // XCD b % 8 sweeps chunk b % 8 of the plan's XCD-interleaved ranges
    const int rng = (P % 8 == 0) ? (bid % 8) * (P / 8) + bid / 8 : bid;
    const int k0 = max(seg[rng], 0), k1 = min(seg[rng + 1], n_items);
    if (k0 >= k1) return;
    const int tid = threadIdx.x, lane = tid & 63;
    const int lw = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave = loader index
    const int g = lane >> 4, r = lane & 15;

    const lds_char *lds = (const lds_char *)smem;
    const int4 *rwin = reinterpret_cast<const int4 *>(smem + kXWin);
    // LDS-DMA with an SGPR base (global_load_lds_dwordx4 v_off, s_base): the
    // only per-lane operand is the byte offset lane*16
    const uint32_t voff = (uint32_t)lane * 16u;
    const uint32_t lds_smem = (uint32_t)(uintptr_t)(lds_char *)(smem);
    const uint32_t lds_wave = lds_smem + (uint32_t)lw * 1024u;
    const uint32_t lds_rwin = lds_smem + (uint32_t)kXWin;
#define SBO_DMA16(sbase, ldst)                                                                          \
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"((const void *)(sbase)),     \
                 "{m0}"(ldst)                                                                           \
                 : "memory")
    // one half-tile stage into LDS slot `sl`: wave 0 brings the item's
    // queries (lanes 0-31 qx, 32-63 qy; with an item's first step only) and
    // the half-tile's coordinates; the A pieces follow -- in a burst for the
    // prologue's stages, else one per row block inside x3_half (a_src, a_dst)
#define SBO_X3_STAGE(akib_, kcf_, h_, qb_, sl_, burst_, first_)                                         \
    do {                                                                                                \
        const uint32_t d_ = lds_smem + (uint32_t)(sl_) * kXSlot;                                        \
        if (lw == 0) {                                                                                  \
            if (first_) {                                                                               \
                if (lane < 32) SBO_DMA16(qx + (int64_t)(qb_) * kBN, d_ + kXA + kXC);                    \
                else SBO_DMA16(qy + (int64_t)(qb_) * kBN - 128, d_ + kXA + kXC);                        \
            }                                                                                           \
            if (lane < 32) SBO_DMA16(kc3 + (uint32_t)(kcf_) + (h_) * (kXC / 4), d_ + kXA);              \
        }                                                                                               \
        const char *s_ = a_base + (uint64_t)((akib_) + (h_) * (kXA / 1024)) * 1024u;                     \
        const uint32_t w_ = lds_wave + (uint32_t)(sl_) * kXSlot;                                        \
        a_src = s_;                                                                                     \
        a_dst = w_;                                                                                     \
        if (burst_)                                                                                     \
            _Pragma("unroll") for (int j = 0; j < kPieces; ++j)                                         \
                SBO_DMA16(s_ + j * kStride, w_ + (uint32_t)(j * kStride));                              \
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
    const char *a_base = ax3 + lw * 1024;
    const char *a_src = ax3;  // this wave's A pieces of the last staged step
    uint32_t a_dst = 0;
    // the record of entry la_e, read when la_e became current (one stage call
    // ahead of its use: the LDS latency off the step top)
    int4 r_cur = rec_at(la_e);
    auto stage = [&](int sl, bool burst) {
        const int4 rr = r_cur;
        XStep s;
        s.I = min(rr.w & 0xffff, nI - 1);
        s.qb = rr.z;
        s.flags = la_h | ((rr.w & kRecFirst) && la_h == 0 ? kFirst : 0) | ((rr.w & kRecLast) && la_h == 1 ? kLast : 0) |
                  kValid;
        s.lv = min((rr.w >> 16) & 3, 2);
        SBO_X3_STAGE(min((uint32_t)rr.x, a_max), rr.y, la_h, rr.z, sl, burst, (s.flags & kFirst) != 0);
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

    // the lane's query in the block
    const int qo = lw * 16 + r;
    f32x4 acc[16], outer[16];
#pragma unroll
    for (int rb = 0; rb < 16; ++rb) {
        acc[rb] = f32x4{};
        outer[rb] = acc[rb];
    }
    double mu = 0.0;
    KPieces kb, nx;
    // the lane's query coordinates of the item whose K* is being built: read
    // from the slot of an item's first step only (its stage alone carries them)
    float xq, yq;
    {
        const lds_char *pq = lds + kXA + kXC;
        xq = lds_f(pq + qo * 4);
        yq = lds_f(pq + (kBN + qo) * 4);
        x3_kstar(lds + kXA, xq, yq, g, cexp, s0.I == nI - 1, kb, mu);
    }
    // deferred outputs of the item finished in the previous step (stored at
    // the top of the next step, before its stage DMA, so that the vmcnt count
    // at the end of every step is the A pieces of one stage)
    bool pend = false, pend_mean = false;
    float pend_s = 0.0f, pend_mu = 0.0f;
    int64_t pend_q = 0;
    int pend_I = 0;
    auto flush = [&]() {
        if (pend && lane < 16 && pend_q < m) {
            part[(int64_t)pend_I * ldp + pend_q] = pend_s;
            if (pend_mean) mean[pend_q] = pend_mu;
        }
        pend = false;
    };
    int cur = 0;
    bool more = true;
    // one half-step; items are whole tiles, so the steps alternate FRESH
    // (first half: chains from zero) and second halves (which may end an item)
    auto half_step = [&](auto fresh_tag) {
        constexpr bool FRESH = decltype(fresh_tag)::value;
        if (FRESH) flush();
        const bool issue = la_e < e_end;
        const int nslot = cur == 0 ? 2 : cur - 1;  // (cur + 2) % 3
        s2 = issue ? stage(nslot, false) : XStep{0, 0, 0, 0};
        // A pieces the staged tile's level needs (plane p = pieces 2p, 2p + 1)
        const int np2 = (kPieces / 3) * (3 - s2.lv);
        if (!issue) a_dst = lds_wave + (uint32_t)nslot * kXSlot;  // a harmless re-stage into the free slot
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
                double u = mu;
                u += __shfl_xor(u, 16);
                u += __shfl_xor(u, 32);
                pend_mu = (float)((double)m0 + u);
            }
            if (nvalid && (s1.flags & kFirst)) mu = 0.0;
        }
        if (nvalid && (s1.flags & kFirst)) {
            xq = lds_f(pqn + qo * 4);
            yq = lds_f(pqn + (kBN + qo) * 4);
        }
        // the body by the tile's level and the next step's (uniform: one
        // branch here, none inside the body's MFMA region)
        if (s0.lv == 2 && nvalid && s1.lv == 2)
            x3_half<FRESH, 2, true>(pa, pcn, xq, yq, g, cexp, msc, kb, acc, outer, nx, mu, voff, a_src, a_dst, np2);
        else if (s0.lv == 2)
            x3_half<FRESH, 2, false>(pa, pcn, xq, yq, g, cexp, msc, kb, acc, outer, nx, mu, voff, a_src, a_dst, np2);
        else if (s0.lv == 1)
            x3_half<FRESH, 1, false>(pa, pcn, xq, yq, g, cexp, msc, kb, acc, outer, nx, mu, voff, a_src, a_dst, np2);
        else
            x3_half<FRESH, 0, false>(pa, pcn, xq, yq, g, cexp, msc, kb, acc, outer, nx, mu, voff, a_src, a_dst, np2);
        if (!FRESH && (s0.flags & kLast)) {
            // item done: column sums of V^2 over its rows (lanes l, l+16, l+32,
            // l+48 hold four row quarters of column l&15 of every block)
            pend = true;
            pend_I = s0.I;
            pend_q = (int64_t)s0.qb * kBN + qo;
            pend_mean = s0.I == nI - 1;
            // four independent f64 chains (element e of every block), then
            // combined: the 64-term sum off one dependent fma chain
            double sq[4] = {};
#pragma unroll
            for (int rb = 0; rb < 16; ++rb)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    sq[e] = fma((double)outer[rb][e], (double)outer[rb][e], sq[e]);
                    outer[rb][e] = 0.0f;
                }
            double sv = (sq[0] + sq[1]) + (sq[2] + sq[3]);
            sv += __shfl_xor(sv, 16);
            sv += __shfl_xor(sv, 32);
            pend_s = (float)sv;
        }
        // retire stage i+1: its queries and coordinates (wave 0) precede its
        // A pieces and were retired one step earlier; leave stage i+2's six A
        // pieces in flight
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
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
#undef SBO_X3_STAGE
#undef SBO_REC_WINDOW
#undef SBO_DMA16
}

// Split the f32 packed operand (tiles T0 .. T1-1, tile_offset layout) into
// the three bf16 planes of the x3 layout: tile T, half h, plane p, row block
// rb, lane l = 16 g + r holds A[16 rb + r][32 h + 8 g + j], j = 0..7, at
// byte T*2*kXA + h*kXA + p*kXPlane + rb*1024 + l*16 + 2j.
__global__ __launch_bounds__(256) void pack_x3_kernel(const float *__restrict__ aug, int64_t T0, int64_t nt,
                                                      char *__restrict__ ax3) {
    const int64_t id = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (id >= nt * 2048) return;
    const int lane = (int)(id & 63), rb = (int)((id >> 6) & 15), h = (int)((id >> 10) & 1);
    const int64_t T = T0 + (id >> 11);
    const int row = rb * 16 + (lane & 15);
    const int k0 = kXH * h + 8 * (lane >> 4);
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
    if (wide) return hipErrorInvalidValue;   // the wide layout (variant 13) is the diagnostic build's
    const int64_t nI = npad / kBM;
    const int64_t T0 = tile_start(I0), T1 = tile_start(nI);
    if (ax3 && T1 > T0) {
        const int64_t th = (T1 - T0) * 2048;
        hipLaunchKernelGGL(pack_x3_kernel, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, s, aug, T0, T1 - T0, ax3);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (!kc3) return hipSuccess;
    const int64_t nkt = npad / kBK;
    hipLaunchKernelGGL(pack_kc3_kernel, dim3((unsigned)((nkt * 256 + 255) / 256)), dim3(256), 0, s, kcoord, nkt, kc3);
    return hipGetLastError();
}

// The product build has no phase stamps (diag/predict_x3_diag.hip): zeros.
hipError_t read_x3_stamps(double *out, int n) {
    for (int j = 0; j < n; ++j) out[j] = 0.0;
    return hipSuccess;
}

hipError_t launch_predict_x3(hipStream_t s, const char *ax3, const float *kc3, const int4 *desc, const int4 *rec,
                             const int *seg, int P, int n_items, int nI, const float *qx, const float *qy, int64_t m,
                             int64_t ldp, float cexp, float m0, float *part, float *mean, int variant) {
    // the largest tile offset a record may name (KiB): keeps every staged address inside ax3
    const int64_t amax = (total_tiles(nI) - 1) * (2 * kXA / 1024);
    if (nI <= 0 || amax > 0xffffffffll) return hipErrorInvalidValue;
    if (variant != 3 && variant != 22) return hipErrorInvalidValue;   // (22: the same kernel, the plan has no levels)
    hipLaunchKernelGGL(predict_x3_kernel, dim3((unsigned)P), dim3(512), 0, s, ax3, kc3, desc, rec, seg, P, n_items, nI,
                       (uint32_t)amax, qx, qy, m, ldp, cexp, m0, part, mean);
    return hipGetLastError();
}

}  // namespace sbo
