// predict_oz.hip -- the precise predictive sweep on the int8 matrix cores
// (round 4; SBO_OPT_PRECISE_KERNEL 1): V = A K*^T with
// A = sf2 L^-1 cut into five and K* into four balanced base-256 int8 digit
// slices, the slice products accumulated EXACTLY in int32 by
// v_mfma_i32_16x16x64_i8 and combined in f64 once per k-tile (an Ozaki-style
// sliced product).
//
// Why: on the mapping node's own box (config/lpsc.yaml:32-37) the fast split
// sweep misses the 1e-5 contract by 40x because it accumulates terms far larger
// than their sum (|A| |k| >> |A k|) in f32; predict_f64.hip
// meets it with f64 MFMA at 0.75 of the 78.6 TF f64 peak, and that pipe has no
// headroom left.  The i8 MFMA runs a 16x16x64 block in the cycles the bf16
// MFMA spends on 16x16x32 (MI355X_MICROARCH.md, matrix cores: 2x bf16 per
// clock) and sums its products exactly, so the rounding the contract cannot
// afford is gone and what is left is the slicing:
//   A: per (16-row block, k-tile) a power of two 2^eA > 1.01 max|A|, the
//      integer XA = rint(A 2^(39 - eA)) (|XA| < 2^39 / 1.01) in five balanced
//      base-256 digits, XA = sum_s D_s 2^(32 - 8 s): the bytes of XA +
//      0x80808080, less 128 but for the top one, so |D_s| <= 128 and |D_0| <=
//      127 (pack_oz_kernel, once per fit / append);
//   K*: in f64 (exp2 of the f64 distance), per (query, k-tile) a power of two
//      2^eK > 1.01 max K*, X = rint(K* 2^(31 - eK)) < 2^31 / 1.01 in four such
//      digits E_u 2^(24 - 8 u), read straight from the mantissa of one f64 add
//      (K* 2^(31 - eK) + 2^52 + 0x808080: the bytes of X + 0x808080, the three
//      lower ones XOR 0x80) in the sweep;
//   product: the 14 pairs (s, u) with s + u <= 4 (u <= 3; the dropped ones sit
//      below 2^-38 of the tile's |A| |K*| scale), level L = s + u chained in one
//      int32 accumulator (no overflow: 64 products of |D| |E| <= 2^14 per pair,
//      at most four pairs per level, < 2^22), the five levels combined in f64
//      per 16x16 block: T = (l0 256 + l1) 2^16 + l2 256 + l3 + round(l4 / 256)
//      (< 2^45; exact but for level 4's last eight bits), V += T 2^(eA + eK - 38).
// (Round 4's first form cut both into base-128 digits by successive rounding:
// 35 bits of A, 28 of K*, the same 14 products, but twelve integer operations
// per K* value to spread 7-bit fields into bytes -- a quarter of the kernel's
// VALU.)  Emulated on the host at N = 8192 on the lpsc box
// (tools/r4_emulate_ozaki.py, base 128): normwise variance error 1.2e-6
// against f64 (the f32-rounded A alone: 6.5e-5); truncated digits or
// three-digit K* miss.
//
// Work items, the tick plan and the persistent walk are predict_f64_kernel's:
// workgroup = 256 rows x 128 queries, eight waves, wave w owns queries
// 16w..16w+15 and all 256 rows as sixteen 16-row blocks of f64 accumulators
// (128 VGPRs).  A stage is half a k-tile's ROWS (128 rows x 64 k x 5 digits =
// 40 KiB, + the eight block exponents, + on the first half the tile's 64
// coordinates and sf2 alpha), double buffered by LDS-DMA, one barrier per
// stage; K*'s digits are built on the first half and kept in registers for the
// second.  Inside a stage the digits are in MFMA fragment order ([digit][block]
// [lane][16 B]), so a lane's A operand of one MFMA is one conflict-free
// ds_read_b128.
#include <cstdint>

#include "sbo_internal.hpp"

namespace sbo {
namespace {

typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr int kOzDigits = 5;                      // base-256 digits of A: XA = rint(A 2^(39 - eA))
constexpr int kOzKDigits = 4;                     // base-256 digits of K*: X = rint(K* 2^(31 - eK))
constexpr int kOzKBits = 31;
constexpr int kOzScale = 38;                      // V += T 2^(eA + eK - 38), T in level-3 units
constexpr int kOzRB = kBM / 16;                   // 16-row blocks per item (per wave)
constexpr int kOzHalfRB = kOzRB / 2;              // blocks per stage
constexpr int kOzPlane = kOzHalfRB * 64 * 16;     // one digit plane of a stage: 8 KiB
constexpr int kOzA = kOzDigits * kOzPlane;        // 40 KiB of digits per stage
constexpr int kOzTileBytes = 2 * kOzA;            // one packed tile: 80 KiB
constexpr int kOzE = 64;                          // the stage's block exponents (8 x int32, padded)
constexpr int kOzC = 3 * kBK * 8 + 2 * kBK * 4;   // per k-tile: x, y, sf2 alpha (f64), x, y (f32) = 2 KiB
constexpr int kOzSlot = kOzA + kOzE + kOzC;
constexpr int kOzWaves = kBN / 16;                // 8
constexpr int kOzThreads = 64 * kOzWaves;
constexpr int kOzDescWin = 64;                    // item descriptors (int4) per 1 KiB window
constexpr int kOzListWin = 512;                   // tile-list entries (u16) per 1 KiB window
constexpr int kOzSmem = 2 * kOzSlot + 4096 + 512; // two stage slots + two descriptor and two list windows + 2^(j/64)
// K*'s digits: X = rint(K* 2^(31 - eK)) + bias, bias = 128 at the three lower
// base-256 positions, by one f64 add of 2^52 + bias (the add rounds to an
// integer and leaves X + bias in the low mantissa bits)
constexpr uint32_t kOzBias = 0x808080u;
constexpr double kOzMagic = 4503599627370496.0 + (double)kOzBias;
static_assert(kOzC == 2048, "a tile's coordinates: two 1 KiB LDS-DMA pieces");
// K* table (SBO_OPT_PRECISE_KERNEL 3): per (query block, k-tile) the sweep's
// digit operands, [wave][digit][lane][16 B] = 32 KiB, then eK per query (128 x
// int32) and the tile's mean terms per query (128 x f64, sum over its 64 k)
constexpr int kKztDigits = kOzWaves * kOzKDigits * 1024;   // 32 KiB
constexpr int kKztE = kKztDigits;                          // + 512 B
constexpr int kKztMu = kKztE + kBN * 4;                    // + 1 KiB
constexpr int kKzt = kKztMu + kBN * 8;                     // 34304 B per (query block, k-tile)
constexpr int kOzSlotT = kOzA + kOzE + kKzt;
constexpr int kOzSmemT = 2 * kOzSlotT + 4096 + 512;
static_assert(kOzSmemT <= 160 * 1024, "two table-mode stage slots must fit the LDS");
static_assert(kOzA % (1024 * kOzWaves) == 0, "stage digits: whole 1 KiB LDS-DMA pieces per wave");

__device__ __forceinline__ i32x4 mfma_i8(i32x4 a, i32x4 b, i32x4 c) {
    return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
}

// 2^u in f64 for the K* digits (u <= 0): u = e + j/64 + r, |r| <= 1/128,
// 2^u = 2^e T[j] P(r) with T[j] = 2^(j/64) from an LDS table and P the degree-5
// the degree-4 Taylor polynomial of 2^r (truncation < (ln2/128)^5 / 120 <
// 2^-44 relative, the table and the Horner steps a few 2^-53): 10 f64
// operations instead of the library exp2's ~30 -- the digits keep 31 bits of
// K* 2^-eK.  Returns T[j] P(r) and sets e (the caller folds 2^e into its scale).
__device__ __forceinline__ double exp2_tab(double u, const double *__restrict__ T, int &e) {
    const double m = rint(u * 64.0);
    const double r = fma(m, -0.015625, u);
    const int mi = (int)m;
    e = mi >> 6;                      // floor(m / 64): arithmetic shift
    const double t = T[mi & 63];
    constexpr double c1 = 0.69314718055994530942, c2 = 0.24022650695910071233, c3 = 0.055504108664821579953,
                     c4 = 0.0096181291076284771620;
    const double p = fma(fma(fma(fma(c4, r, c3), r, c2), r, c1), r, 1.0);
    return t * p;
}

// K*'s four digit operands for this lane's 16 k (k = 16 g + j, g = lane >> 4)
// and its query, from the tile's coordinates in LDS: Y = rint(K* 2^(31 - eK))
// + bias as the low 32 bits of K* 2^(31 - eK) + 2^52 + bias (f64, exact); its
// bytes are the digits, the top one in byte 3 and the three lower ones XOR
// 0x80 (byte - 128 in two's complement) -- transposed four k at a time so that
// digit u of k = 16 g + j is byte j of kd[u].  The per-(query, tile) exponent
// eK needs the max over all 64 k: the four lanes l, l ^ 16, l ^ 32, l ^ 48
// hold them; the max K* is the min distance's, so pass 1 is the f32 distance
// alone (the stored f32 coordinates) and one v_exp_f32 per lane.  Four digits
// (31 bits) suffice for K*: its f32 rounding (24 bits) alone moved the lpsc
// box's variance by only 2.6e-6 (tools/r4_emulate_ozaki.py), against 6.5e-5
// for A.  On the last row block (mean) also mu += K* sf2 alpha.
// pass 1 of kstar_digits: the smallest f32 squared distance from the query
// to the tile's 64 points (this lane's 16, then the four lanes of a query)
__device__ __forceinline__ float kstar_dmin(const char *__restrict__ pc, int g, double xq, double yq) {
    const float *px32 = reinterpret_cast<const float *>(pc + kBK * 24) + 16 * g;
    const float *py32 = reinterpret_cast<const float *>(pc + kBK * 28) + 16 * g;
    const float xqf = (float)xq, yqf = (float)yq;
    float dmin = 3.0e38f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const float dx = px32[j] - xqf, dy = py32[j] - yqf;
        dmin = fminf(dmin, fmaf(dy, dy, dx * dx));
    }
    dmin = fminf(dmin, __shfl_xor(dmin, 16));
    dmin = fminf(dmin, __shfl_xor(dmin, 32));
    return dmin;
}
// the exponent: 2^eK > 1.01 kmax, so K* 2^-eK < 0.99 and the top digit stays <= 127
__device__ __forceinline__ int kstar_exp(float dmin, double cexp) {
    const float kmax = __builtin_amdgcn_exp2f((float)cexp * dmin);
    int e = 0;
    (void)frexpf(kmax * 1.01f, &e);
    return kmax > 0.0f ? e : 0;
}
// pass 2: the digits under a given exponent eK
template <bool MEAN>
__device__ __forceinline__ void kstar_digits_e(const char *__restrict__ pc, const double *__restrict__ T2, int g,
                                               double xq, double yq, double cexp, int eK, i32x4 (&kd)[kOzKDigits],
                                               double &mu) {
    const double *px = reinterpret_cast<const double *>(pc) + 16 * g;
    const double *py = reinterpret_cast<const double *>(pc + kBK * 8) + 16 * g;
    const double *pa = reinterpret_cast<const double *>(pc + kBK * 16) + 16 * g;
    const int esc = kOzKBits - eK;
#pragma unroll
    for (int m4 = 0; m4 < 4; ++m4) {
        uint32_t lo[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int j = 4 * m4 + i;
            const double dx = px[j] - xq, dy = py[j] - yq;
            int ex;
            const double kt = exp2_tab(cexp * fma(dy, dy, dx * dx), T2, ex);   // K* = kt 2^ex
            if (MEAN) mu = fma(ldexp(kt, ex), pa[j], mu);
            const uint32_t Y = (uint32_t)__builtin_bit_cast(uint64_t, ldexp(kt, ex + esc) + kOzMagic);
            lo[i] = Y ^ 0x00808080u;   // top digit in byte 3; the lower ones byte - 128
        }
        // 4 x 4 byte transpose: byte i of the dword for digit u = byte (3 - u) of lo[i]
        const uint32_t p01a = __builtin_amdgcn_perm(lo[1], lo[0], 0x05010400u);   // lo0.b0 lo1.b0 lo0.b1 lo1.b1
        const uint32_t p01b = __builtin_amdgcn_perm(lo[1], lo[0], 0x07030602u);   // lo0.b2 lo1.b2 lo0.b3 lo1.b3
        const uint32_t p23a = __builtin_amdgcn_perm(lo[3], lo[2], 0x05010400u);
        const uint32_t p23b = __builtin_amdgcn_perm(lo[3], lo[2], 0x07030602u);
        kd[3][m4] = (int)__builtin_amdgcn_perm(p23a, p01a, 0x05040100u);          // bytes 0 of lo0..lo3
        kd[2][m4] = (int)__builtin_amdgcn_perm(p23a, p01a, 0x07060302u);          // bytes 1
        kd[1][m4] = (int)__builtin_amdgcn_perm(p23b, p01b, 0x05040100u);          // bytes 2
        kd[0][m4] = (int)__builtin_amdgcn_perm(p23b, p01b, 0x07060302u);          // bytes 3: the top digit
    }
}
// pass 1 (the exponent from an f32 estimate of the largest K*: the min
// distance, v_exp_f32, a few ulp -- the 1.01 margin covers it), so that pass
// 2 can cut each f64 K* into digits as soon as it is computed (four live at a
// time, not sixteen)
template <bool MEAN>
__device__ __forceinline__ void kstar_digits(const char *__restrict__ pc, const double *__restrict__ T2, int g,
                                             double xq, double yq, double cexp, i32x4 (&kd)[kOzKDigits], int &eK,
                                             double &mu) {
    eK = kstar_exp(kstar_dmin(pc, g, xq, yq), cexp);
    kstar_digits_e<MEAN>(pc, T2, g, xq, yq, cexp, eK, kd, mu);
}

// The 14 digit products of one 16x16 block (A digit s, K* digit u, s + u <=
// 4, u <= 3), combined and added to acc scaled by 2^(eA + eK - 38): level 4 is
// folded into level 3 rounded to a level-3 unit (2^-39 of the tile's scale
// 2^(eA + eK)), the rest exactly: T = (l0 256 + l1) 2^16 + l2 256 + l3 +
// [l4 / 256] in level-3 units, two conversions and two f64 operations per value.
__device__ __forceinline__ void block_products(const i32x4 (&ad)[kOzDigits], const i32x4 (&kd)[kOzKDigits],
                                               double S, f64x4 &acc) {
    // ordered by A digit (each ad[s] dies after its group; the int32 sums are
    // exact, so the order does not change the result)
    const i32x4 z = {0, 0, 0, 0};
    i32x4 l0 = mfma_i8(ad[0], kd[0], z);
    i32x4 l1 = mfma_i8(ad[0], kd[1], z);
    i32x4 l2 = mfma_i8(ad[0], kd[2], z);
    i32x4 l3 = mfma_i8(ad[0], kd[3], z);
    l1 = mfma_i8(ad[1], kd[0], l1);
    l2 = mfma_i8(ad[1], kd[1], l2);
    l3 = mfma_i8(ad[1], kd[2], l3);
    i32x4 l4 = mfma_i8(ad[1], kd[3], z);
    l2 = mfma_i8(ad[2], kd[0], l2);
    l3 = mfma_i8(ad[2], kd[1], l3);
    l4 = mfma_i8(ad[2], kd[2], l4);
    l3 = mfma_i8(ad[3], kd[0], l3);
    l4 = mfma_i8(ad[3], kd[1], l4);
    l4 = mfma_i8(ad[4], kd[0], l4);
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        const int h01 = l0[v] * 256 + l1[v];                      // |.| < 2^29
        const int h23 = l2[v] * 256 + l3[v] + ((l4[v] + 128) >> 8);  // |.| < 2^30
        const double t = fma((double)h01, 65536.0, (double)h23);  // exact, < 2^45
        acc[v] = fma(t, S, acc[v]);
    }
}

// One stage: the eight 16-row blocks of the staged half, all in one code path
// per half (the accumulators are indexed statically).
template <int H>
__device__ __forceinline__ void stage_blocks(const char *__restrict__ slot, int lane, const i32x4 (&kd)[kOzKDigits],
                                             int eK, f64x4 (&acc)[kOzRB]) {
    const int *eA = reinterpret_cast<const int *>(slot + kOzA);
    const i32x4 *pa = reinterpret_cast<const i32x4 *>(slot) + lane;
    // (prefetching the next block's digits here measured slower: the extra
    // 20 registers spill; SBO_OPT_PRECISE_KERNEL A/B, round 4)
#pragma unroll
    for (int rb = 0; rb < kOzHalfRB; ++rb) {
        i32x4 ad[kOzDigits];
#pragma unroll
        for (int s = 0; s < kOzDigits; ++s) ad[s] = pa[s * (kOzPlane / 16) + rb * 64];
        const double S = ldexp(1.0, __builtin_amdgcn_readfirstlane(eA[rb]) + eK - kOzScale);
        block_products(ad, kd, S, acc[H * kOzHalfRB + rb]);
    }
}

// Every wave builds its K* digits at the top of a tile's first stage.  (A/B,
// round 4: staggering the two waves of a SIMD -- waves 4-7 building the next
// tile's digits a stage early, so that one wave's VALU work overlaps the
// other's products -- needs a second digit set; at 87 spilled registers it
// ran at 4517 ms against 2296 on the lpsc box and was dropped.)
// MODE 0: K*'s digits built in the sweep; 2 (TABLE): read from the K* table
// (kstar_table_kernel, one pass per query block and k-tile instead of one per
// row block), staged with each tile's first stage; 1 (diagnostic build only,
// wrong results): not built -- the bound on what the K* work costs the sweep.
template <int MODE>
__global__ __launch_bounds__(kOzThreads, 1) void predict_oz_kernel(
    const char *__restrict__ aoz, const int *__restrict__ eoz, const char *__restrict__ koz,
    const int4 *__restrict__ desc, const unsigned short *__restrict__ tl, const int *__restrict__ seg, int P,
    int n_items, int nI, const float *__restrict__ qx, const float *__restrict__ qy, int64_t m, int64_t ldp,
    double cexp, double m0, double *__restrict__ part, double *__restrict__ mean, const char *__restrict__ kzt) {
    // (diagnostic build only, wrong results: MODE 3 = TABLE without any stage
    // DMA -- the compute bound; 4 = TABLE without the table's DMA)
    constexpr bool NOKSTAR = MODE == 1, TABLE = MODE >= 2, DMA_A = MODE != 3, DMA_T = MODE == 2;
    constexpr int kSlot = TABLE ? kOzSlotT : kOzSlot;
    __shared__ __attribute__((aligned(16))) char smem[TABLE ? kOzSmemT : kOzSmem];
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
    const int4 *dwin = reinterpret_cast<const int4 *>(smem + 2 * kSlot);
    const unsigned short *lwin = reinterpret_cast<const unsigned short *>(smem + 2 * kSlot + 2048);
    double *T2 = reinterpret_cast<double *>(smem + 2 * kSlot + 4096);
    if (tid < 64) T2[tid] = exp2((double)tid * 0.015625);   // (visible after the prologue's barriers)

    // LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave instruction, lane
    // linear), issued from inline asm as in predict_f64_kernel: every wave
    // moves 5 KiB of each 40 KiB stage; wave 0 lanes 0-1 the stage's eight
    // block exponents, wave 1 the tile's coordinates on its first half.
    typedef __attribute__((address_space(3))) char lds_char;
    const uint32_t lds_smem = (uint32_t)(uintptr_t)(lds_char *)(smem);
    const uint32_t lds_wave = lds_smem + (uint32_t)__builtin_amdgcn_readfirstlane(wave) * 1024u;
    const uint32_t lds_dwin = lds_smem + 2u * kSlot;
    const uint32_t lds_lwin = lds_dwin + 2048u;
    const char *gA = aoz + wave * 1024 + lane * 16;
    const char *gE = reinterpret_cast<const char *>(eoz) + lane * 16;
    const char *gC = koz + lane * 16;
    const char *gD = reinterpret_cast<const char *>(desc) + lane * 16;
    const char *gL = reinterpret_cast<const char *>(tl) + lane * 16;
    const char *gZ = kzt + lane * 16;
    const int wave_u = __builtin_amdgcn_readfirstlane(wave);
    const int nkt = kTilesPerRowBlockStep * nI;
#define SBO_OZ_DMA16(gsrc, ldst)                                                                         \
    do {                                                                                                 \
        uint32_t keep_;                                                                                  \
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t" \
                     "s_mov_b32 m0, %0"                                                                  \
                     : "=&s"(keep_)                                                                      \
                     : "v"(gsrc), "s"(ldst)                                                              \
                     : "memory");                                                                        \
    } while (0)
    // stage (packed tile T_, row half h_) into slot buf, with the coordinates
    // of k-tile kt_ (TABLE: its K* table piece for query block qb_; none: kt_ < 0)
#define SBO_OZ_STAGE(T_, kt_, h_, buf, qb_)                                                              \
    do {                                                                                                 \
        const char *s_ = gA + (int64_t)(T_) * kOzTileBytes + (h_) * kOzA;                                \
        const uint32_t d_ = __builtin_amdgcn_readfirstlane(lds_wave + (uint32_t)(buf) * kSlot);          \
        if (DMA_A)                                                                                       \
            _Pragma("unroll") for (int j_ = 0; j_ < kOzA / (1024 * kOzWaves); ++j_)                      \
                SBO_OZ_DMA16(s_ + j_ * kOzWaves * 1024, d_ + (uint32_t)(j_ * kOzWaves * 1024));          \
        if (DMA_A && wave == 0 && lane < 2)                                                              \
            SBO_OZ_DMA16(gE + (int64_t)(T_) * 64 + (h_) * 32,                                            \
                         __builtin_amdgcn_readfirstlane(lds_smem + (uint32_t)((buf) * kSlot + kOzA)));       \
        if (TABLE) {                                                                                     \
            if (DMA_T && (kt_) >= 0) {                                                                   \
                const char *z_ = gZ + ((int64_t)(qb_) * nkt + (kt_)) * kKzt;                              \
                const uint32_t zd_ = __builtin_amdgcn_readfirstlane(lds_smem + (uint32_t)((buf) * kSlot + kOzA + kOzE)); \
                _Pragma("unroll") for (int u_ = 0; u_ < kOzKDigits; ++u_)                                \
                    SBO_OZ_DMA16(z_ + wave * 4096 + u_ * 1024, zd_ + (uint32_t)(wave_u * 4096 + u_ * 1024)); \
                if (wave == 0 && lane < 32) SBO_OZ_DMA16(z_ + kKztE, zd_ + (uint32_t)kKztE);             \
                if (wave == 1) SBO_OZ_DMA16(z_ + kKztMu, zd_ + (uint32_t)kKztMu);                        \
            }                                                                                            \
        } else if ((kt_) >= 0 && (wave == 1 || wave == 3))                                               \
            SBO_OZ_DMA16(gC + (int64_t)(kt_) * kOzC + (wave == 3 ? 1024 : 0),                            \
                         __builtin_amdgcn_readfirstlane(lds_smem + (uint32_t)((buf) * kSlot + kOzA + kOzE +     \
                                                                              (wave == 3 ? 1024 : 0))));     \
    } while (0)
#define SBO_OZ_DESC_WINDOW(w_)                                                                           \
    do {                                                                                                 \
        if (wave == 1) SBO_OZ_DMA16(gD + (int64_t)(w_) * 1024, lds_dwin + (uint32_t)((w_) & 1) * 1024u); \
    } while (0)
#define SBO_OZ_LIST_WINDOW(w_)                                                                           \
    do {                                                                                                 \
        if (wave == 2) SBO_OZ_DMA16(gL + (int64_t)(w_) * 1024, lds_lwin + (uint32_t)((w_) & 1) * 1024u); \
    } while (0)
    auto desc_at = [&](int k) {  // wave-uniform descriptor from its (loaded) window
        const int4 d = dwin[((k / kOzDescWin) & 1) * kOzDescWin + k % kOzDescWin];
        const int I = min(max(__builtin_amdgcn_readfirstlane(d.x), 0), nI - 1);
        return make_int4(I, __builtin_amdgcn_readfirstlane(d.y), __builtin_amdgcn_readfirstlane(d.z),
                         __builtin_amdgcn_readfirstlane(d.w));
    };
    auto entry_off = [](const int4 &d) {
        return (uint64_t)(uint32_t)d.z | ((uint64_t)((uint32_t)d.w >> 16) << 32);
    };
    auto list_at = [&](uint64_t e, int I) {  // the k-tile of tile-list entry e (level code ignored)
        const int t = __builtin_amdgcn_readfirstlane((int)lwin[((e / kOzListWin) & 1) * kOzListWin + e % kOzListWin]) &
                      ((1 << kLevelShift) - 1);
        return min(t, kTilesPerRowBlockStep * (I + 1) - 1);
    };

    // ---- prologue: the first two windows of each kind, the first stage
    SBO_OZ_DESC_WINDOW(k0 / kOzDescWin);
    SBO_OZ_DESC_WINDOW(k0 / kOzDescWin + 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int4 dc = desc_at(k0);
    uint64_t e = entry_off(dc);
    SBO_OZ_LIST_WINDOW(e / kOzListWin);
    SBO_OZ_LIST_WINDOW(e / kOzListWin + 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int t = list_at(e, dc.x);
    SBO_OZ_STAGE(tile_start(dc.x) + t, t, 0, 0, dc.y);
    int64_t q = (int64_t)dc.y * kBN + wave * 16 + r;
    double xq = (double)qx[q < m ? q : m - 1], yq = (double)qy[q < m ? q : m - 1];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    f64x4 acc[kOzRB];
#pragma unroll
    for (int rb = 0; rb < kOzRB; ++rb) acc[rb] = f64x4{0.0, 0.0, 0.0, 0.0};
    i32x4 kd[kOzKDigits];
    int eK = 0;
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
                if (kn % kOzDescWin == 0) SBO_OZ_DESC_WINDOW(kn / kOzDescWin + 1);
                const int64_t qn = (int64_t)dn.y * kBN + wave * 16 + r;
                xqn = (double)qx[qn < m ? qn : m - 1];
                yqn = (double)qy[qn < m ? qn : m - 1];
            }
            if (hn == 0) {
                const uint64_t en = e + 1;
                if (en % kOzListWin == 0) SBO_OZ_LIST_WINDOW(en / kOzListWin + 1);
                tn = list_at(en, dn.x);
            }
            SBO_OZ_STAGE(tile_start(dn.x) + tn, hn == 0 ? tn : -1, hn, cur ^ 1, dn.y);
        }
        const char *slot = smem + cur * kSlot;
        const int I = dc.x;
        if (h == 0) {
            if (NOKSTAR) {
#pragma unroll
                for (int u = 0; u < kOzKDigits; ++u) kd[u] = i32x4{lane + u, lane ^ u, 3 * u, t};
                eK = -8;
            } else if (TABLE) {
                const char *tz = slot + kOzA + kOzE;
#pragma unroll
                for (int u = 0; u < kOzKDigits; ++u)
                    kd[u] = *reinterpret_cast<const i32x4 *>(tz + wave * 4096 + u * 1024 + lane * 16);
                eK = *reinterpret_cast<const int *>(tz + kKztE + (wave * 16 + r) * 4);
                // the tile's mean terms (summed over its 64 k) once per query
                if (I == nI - 1 && g == 0) mu += *reinterpret_cast<const double *>(tz + kKztMu + (wave * 16 + r) * 8);
            } else if (I == nI - 1)
                kstar_digits<true>(slot + kOzA + kOzE, T2, g, xq, yq, cexp, kd, eK, mu);
            else
                kstar_digits<false>(slot + kOzA + kOzE, T2, g, xq, yq, cexp, kd, eK, mu);
            stage_blocks<0>(slot, lane, kd, eK, acc);
        } else {
            stage_blocks<1>(slot, lane, kd, eK, acc);
        }
        if (h == 1 && j == cnt - 1) {
            // item done: column sums of V^2 over its 256 rows; lane l holds
            // rows 4 (l >> 4) + v of every 16-row block, column l & 15
            double sum = 0.0;
#pragma unroll
            for (int rb = 0; rb < kOzRB; ++rb) {
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
#undef SBO_OZ_STAGE
#undef SBO_OZ_DESC_WINDOW
#undef SBO_OZ_LIST_WINDOW
#undef SBO_OZ_DMA16
}

#ifdef SBO_DIAG
// SBO_OPT_PRECISE_KERNEL 5 (round 5; diagnostic build only -- measured no
// faster than kernel 3): kernel 3 with a deeper stream.  Kernel
// 3 stages one half-tile ahead (two slots of A + the K* table piece, 150 KiB),
// so each 40 KiB stage has one stage of MFMA time (~1.7 us) to arrive -- at
// 114 KiB per tile a CU needs ~38 GB/s for that, beyond what the L2-missing
// part of the stream delivers per CU (MI355X_MICROARCH.md, gather rates: 23-34
// GB/s per CU from HBM / the Infinity Cache at ~72 KiB in flight).  Here A is
// staged a whole TILE ahead in three slots (the stage s + 2 into the slot stage
// s - 1 read), and the K* table piece -- read into registers once per tile at
// its first half -- is single-buffered per wave: each wave DMAs its own
// digits, eK (lanes < 4) and mean terms (lanes < 8) of the next tile right
// after reading the current one, two stages before use.  3 x 41 KiB + 33.5
// KiB + windows = 158 KiB of LDS.  The waits are counted: at the end of a
// first-half stage vmcnt(A group + table group) leaves the next tile's
// pieces in flight, at the end of a second-half stage vmcnt(A group); anything
// issued earlier (windows, the previous stage's groups) is complete there.
// Products, digits and sums are kernel 3's: results bitwise equal.
// a wave-uniform pointer the compiler cannot prove uniform, into SGPRs
__device__ __forceinline__ const char *sgpr_ptr(const char *p) {
    const uint64_t v = (uint64_t)(uintptr_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return reinterpret_cast<const char *>((uintptr_t)(((uint64_t)hi << 32) | lo));
}
constexpr int kOz3Slot = kOzA + kOzE;                       // A digits + block exponents
constexpr int kOz3Table = 3 * kOz3Slot;                     // the K* table piece (per-wave parts)
constexpr int kOz3Win = kOz3Table + kKzt;                   // descriptor + list windows
constexpr int kOz3Smem = kOz3Win + 4096;
constexpr int kOz3AGroup = kOzA / (1024 * kOzWaves) + 1;    // A DMA instructions per wave per stage (5 + exponents)
constexpr int kOz3TGroup = kOzKDigits + 2;                  // table DMA instructions per wave per tile (6)
static_assert(kOz3Smem <= 160 * 1024, "three A slots and one table piece must fit the LDS");
static_assert(kOz3AGroup == 6 && kOz3TGroup == 6, "the vmcnt immediates below");

__global__ __launch_bounds__(kOzThreads, 1) void predict_oz3_kernel(
    const char *__restrict__ aoz, const int *__restrict__ eoz, const int4 *__restrict__ desc,
    const unsigned short *__restrict__ tl, const int *__restrict__ seg, int P, int n_items, int nI, int64_t m,
    int64_t ldp, double m0, double *__restrict__ part, double *__restrict__ mean, const char *__restrict__ kzt) {
    __shared__ __attribute__((aligned(16))) char smem[kOz3Smem];
    const int bid = blockIdx.x;
    const int rng = (P % 8 == 0) ? (bid % 8) * (P / 8) + bid / 8 : bid;
    const int k0 = max(seg[rng], 0), k1 = min(seg[rng + 1], n_items);
    if (k0 >= k1) return;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int r = lane & 15;
    const int g = lane >> 4;
    const int4 *dwin = reinterpret_cast<const int4 *>(smem + kOz3Win);
    const unsigned short *lwin = reinterpret_cast<const unsigned short *>(smem + kOz3Win + 2048);
    typedef __attribute__((address_space(3))) char lds_char;
    const uint32_t lds_smem = (uint32_t)(uintptr_t)(lds_char *)(smem);
    const int wave_u = __builtin_amdgcn_readfirstlane(wave);
    const uint32_t lds_wave = lds_smem + (uint32_t)wave_u * 1024u;
    const uint32_t lds_dwin = lds_smem + kOz3Win;
    const uint32_t lds_lwin = lds_dwin + 2048u;
    const uint32_t lds_tab = lds_smem + kOz3Table;
    const int nkt = kTilesPerRowBlockStep * nI;
    // LDS-DMA with an SGPR base (global_load_lds_dwordx4 v_off, s_base), as in
    // predict_x3.hip: the only per-lane operand is the byte offset lane * 16,
    // so no 64-bit per-lane address competes with the accumulators for VGPRs
    // (a spilled address's reload waits for vmcnt(0), which would drain the
    // stream this kernel keeps in flight); the partial pieces run under a
    // wave-uniform EXEC mask, so every wave issues the same count.
    const uint32_t voff = (uint32_t)lane * 16u;
    const char *sA = aoz + (int64_t)wave_u * 1024;
    const char *sE = reinterpret_cast<const char *>(eoz);
    const char *sD = reinterpret_cast<const char *>(desc);
    const char *sL = reinterpret_cast<const char *>(tl);
    // (the windows: wave 1 the descriptors, wave 2 the list; masks in SGPRs)
    const uint64_t win_mask1 = (uint64_t)0 - (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(wave == 1 ? 1 : 0);
    const uint64_t win_mask2 = (uint64_t)0 - (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(wave == 2 ? 1 : 0);
#define SBO_OZ3_DMA16(sbase, ldst)                                                                       \
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"((const void *)sgpr_ptr(sbase)), \
                 "{m0}"(ldst)                                                                           \
                 : "memory")
#define SBO_OZ3_DMA16M(sbase, ldst, mask)                                                                \
    do {                                                                                                 \
        uint64_t sv_;                                                                                    \
        asm volatile("s_mov_b64 %0, exec\n\ts_and_b64 exec, exec, %4\n\ts_nop 0\n\t"                     \
                     "global_load_lds_dwordx4 %1, %2\n\ts_mov_b64 exec, %0"                              \
                     : "=&s"(sv_)                                                                        \
                     : "v"(voff), "s"((const void *)sgpr_ptr(sbase)), "{m0}"(ldst), "s"((uint64_t)(mask)) \
                     : "memory", "scc");                                                                 \
    } while (0)
    // half h_ of packed tile T_ into A slot sl_ (the exponents by every wave's
    // lanes 0-1: the same 32 B, so the per-wave group counts are uniform)
#define SBO_OZ3_A(T_, h_, sl_)                                                                           \
    do {                                                                                                 \
        const char *s_ = sA + (int64_t)(T_) * kOzTileBytes + (h_) * kOzA;                                \
        const uint32_t d_ = __builtin_amdgcn_readfirstlane(lds_wave + (uint32_t)(sl_) * kOz3Slot);       \
        _Pragma("unroll") for (int j_ = 0; j_ < kOz3AGroup - 1; ++j_)                                    \
            SBO_OZ3_DMA16(s_ + j_ * kOzWaves * 1024, d_ + (uint32_t)(j_ * kOzWaves * 1024));             \
        SBO_OZ3_DMA16M(sE + (int64_t)(T_) * 64 + (h_) * 32,                                              \
                       __builtin_amdgcn_readfirstlane(lds_smem + (uint32_t)((sl_) * kOz3Slot + kOzA)), 0x3ull); \
    } while (0)
    // this wave's part of the K* table piece of (query block qb_, k-tile kt_)
#define SBO_OZ3_TABLE(kt_, qb_)                                                                          \
    do {                                                                                                 \
        const char *z_ = kzt + ((int64_t)(qb_) * nkt + (kt_)) * kKzt;                                     \
        _Pragma("unroll") for (int u_ = 0; u_ < kOzKDigits; ++u_)                                        \
            SBO_OZ3_DMA16(z_ + wave_u * 4096 + u_ * 1024, lds_tab + (uint32_t)(wave_u * 4096 + u_ * 1024)); \
        SBO_OZ3_DMA16M(z_ + kKztE + wave_u * 64, lds_tab + (uint32_t)(kKztE + wave_u * 64), 0xfull);     \
        SBO_OZ3_DMA16M(z_ + kKztMu + wave_u * 128, lds_tab + (uint32_t)(kKztMu + wave_u * 128), 0xffull); \
    } while (0)
#define SBO_OZ3_DESC_WINDOW(w_)                                                                          \
    SBO_OZ3_DMA16M(sD + (int64_t)(w_) * 1024, lds_dwin + (uint32_t)((w_) & 1) * 1024u, win_mask1)
#define SBO_OZ3_LIST_WINDOW(w_)                                                                          \
    SBO_OZ3_DMA16M(sL + (int64_t)(w_) * 1024, lds_lwin + (uint32_t)((w_) & 1) * 1024u, win_mask2)
    auto desc_at = [&](int k) {
        const int4 d = dwin[((k / kOzDescWin) & 1) * kOzDescWin + k % kOzDescWin];
        const int I = min(max(__builtin_amdgcn_readfirstlane(d.x), 0), nI - 1);
        return make_int4(I, __builtin_amdgcn_readfirstlane(d.y), __builtin_amdgcn_readfirstlane(d.z),
                         __builtin_amdgcn_readfirstlane(d.w));
    };
    auto entry_off = [](const int4 &d) {
        return (uint64_t)(uint32_t)d.z | ((uint64_t)((uint32_t)d.w >> 16) << 32);
    };
    auto list_at = [&](uint64_t e, int I) {
        const int t = __builtin_amdgcn_readfirstlane((int)lwin[((e / kOzListWin) & 1) * kOzListWin + e % kOzListWin]) &
                      ((1 << kLevelShift) - 1);
        return min(t, kTilesPerRowBlockStep * (I + 1) - 1);
    };

    // ---- prologue: windows, the first tile (both halves and its table piece)
    SBO_OZ3_DESC_WINDOW(k0 / kOzDescWin);
    SBO_OZ3_DESC_WINDOW(k0 / kOzDescWin + 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // the current tile (k, j: item and its j-th tile; e: its tile-list entry)
    int4 dc = desc_at(k0);
    uint64_t e = entry_off(dc);
    SBO_OZ3_LIST_WINDOW(e / kOzListWin);
    SBO_OZ3_LIST_WINDOW(e / kOzListWin + 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int j = 0;
    const int t = list_at(e, dc.x);
    SBO_OZ3_TABLE(t, dc.y);
    SBO_OZ3_A(tile_start(dc.x) + t, 0, 0);
    SBO_OZ3_A(tile_start(dc.x) + t, 1, 1);
    // the next tile (kN, jN, eN, tN, dN), valid while kN < k1; its windows are
    // requested as it enters them (each is read only after a later barrier)
    int kN = k0, jN = 1, tN = 0;
    uint64_t eN = e + 1;
    int4 dN = dc;
    auto advance = [&]() {
        if (jN >= (dN.w & 0xffff)) {
            ++kN;
            jN = 0;
            if (kN < k1) {
                dN = desc_at(kN);
                if (kN % kOzDescWin == 0) SBO_OZ3_DESC_WINDOW(kN / kOzDescWin + 1);
            }
        }
        if (kN < k1) {
            if (eN % kOzListWin == 0) SBO_OZ3_LIST_WINDOW(eN / kOzListWin + 1);
            tN = list_at(eN, dN.x);
        }
    };
    advance();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    f64x4 acc[kOzRB];
#pragma unroll
    for (int rb = 0; rb < kOzRB; ++rb) acc[rb] = f64x4{0.0, 0.0, 0.0, 0.0};
    i32x4 kd[kOzKDigits];
    int eK = 0;
    double mu = 0.0;
    int64_t q = (int64_t)dc.y * kBN + wave * 16 + r;
    int sl = 0, h = 0;
    for (;;) {
        const bool more = kN < k1;
        const char *slot = smem + sl * kOz3Slot;
        const int sl2 = sl == 0 ? 2 : sl - 1;   // (sl + 2) % 3: the slot stage s - 1 read
        const int I = dc.x;
        if (more) SBO_OZ3_A(tile_start(dN.x) + tN, h, sl2);
        if (h == 0) {
            // this tile's K* digits into registers, then (the wave's reads
            // done) the next tile's table piece into the same bytes
            const char *tz = smem + kOz3Table;
#pragma unroll
            for (int u = 0; u < kOzKDigits; ++u)
                kd[u] = *reinterpret_cast<const i32x4 *>(tz + wave * 4096 + u * 1024 + lane * 16);
            eK = *reinterpret_cast<const int *>(tz + kKztE + (wave * 16 + r) * 4);
            if (I == nI - 1 && g == 0) mu += *reinterpret_cast<const double *>(tz + kKztMu + (wave * 16 + r) * 8);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (more) SBO_OZ3_TABLE(tN, dN.y);
            stage_blocks<0>(slot, lane, kd, eK, acc);
        } else {
            stage_blocks<1>(slot, lane, kd, eK, acc);
        }
        if (h == 1 && j == (dc.w & 0xffff) - 1) {
            // item done: column sums of V^2 over its 256 rows
            double sum = 0.0;
#pragma unroll
            for (int rb = 0; rb < kOzRB; ++rb) {
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
        // the next tile's pieces issued in this stage may stay in flight; what
        // was issued before them (the stage after this one) has landed
        if (!more)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else if (h == 0)
            asm volatile("s_waitcnt vmcnt(12)" ::: "memory");   // kOz3AGroup + kOz3TGroup
        else
            asm volatile("s_waitcnt vmcnt(6)" ::: "memory");    // kOz3AGroup
        __syncthreads();
        if (h == 1) {
            if (!more) break;
            j = jN;
            q = (int64_t)dN.y * kBN + wave * 16 + r;
            dc = dN;
            ++jN;
            ++eN;
            advance();
        }
        h ^= 1;
        sl = sl == 2 ? 0 : sl + 1;
    }
#undef SBO_OZ3_A
#undef SBO_OZ3_TABLE
#undef SBO_OZ3_DESC_WINDOW
#undef SBO_OZ3_LIST_WINDOW
#undef SBO_OZ3_DMA16
#undef SBO_OZ3_DMA16M
}

#endif  // SBO_DIAG

// The K* table of nq query blocks (SBO_OPT_PRECISE_KERNEL 3): one workgroup per
// (k-tile t, query block), each wave its 16 queries' digit operands exactly as
// the sweep builds them (kstar_digits), eK per query and the tile's mean terms
// per query -- once per (query block, k-tile) instead of once per row block
// that reads the tile (up to nI times).  grid = (nkt, nq).
__global__ __launch_bounds__(kOzThreads) void kstar_table_kernel(const char *__restrict__ koz,
                                                                 const float *__restrict__ qx,
                                                                 const float *__restrict__ qy, int64_t m, int nkt,
                                                                 int64_t nq, double cexp, char *__restrict__ kzt) {
    __shared__ double T2[64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, r = lane & 15;
    if (tid < 64) T2[tid] = exp2((double)tid * 0.015625);
    __syncthreads();
    const int t = blockIdx.x;
    for (int64_t qb = blockIdx.y; qb < nq; qb += gridDim.y) {   // (grid.y capped at kMaxGridY)
        const int64_t q = qb * kBN + wave * 16 + r;
        const double xq = (double)qx[q < m ? q : m - 1], yq = (double)qy[q < m ? q : m - 1];
        i32x4 kd[kOzKDigits];
        int eK = 0;
        double mu = 0.0;
        kstar_digits<true>(koz + (int64_t)t * kOzC, T2, g, xq, yq, cexp, kd, eK, mu);
        mu += __shfl_xor(mu, 16);
        mu += __shfl_xor(mu, 32);
        char *out = kzt + (qb * nkt + t) * (int64_t)kKzt;
#pragma unroll
        for (int u = 0; u < kOzKDigits; ++u)
            *reinterpret_cast<i32x4 *>(out + wave * 4096 + u * 1024 + lane * 16) = kd[u];
        if (g == 0) {
            reinterpret_cast<int *>(out + kKztE)[wave * 16 + r] = eK;
            reinterpret_cast<double *>(out + kKztMu)[wave * 16 + r] = mu;
        }
    }
}

// A = sf2 L^-1 (from the fit's f64 inverse, lower, column-major, lda ld) into
// int8 digit tiles for row blocks I >= I0: tile (I, t) at tile_start(I) + t,
// 80 KiB = [row half h][digit s][16-row block rb][lane l][byte j], element
// (row 128 h + 16 rb + (l & 15), k = 64 t + 16 (l >> 4) + j); the exponent of
// each 16-row block at eoz[16 (tile_start(I) + t) + 8 h + rb].  One workgroup
// per tile, one thread per row: its 64 values, the block max by a 16-lane
// reduction, then the digits of 16 consecutive k packed into one 16-B store
// per (digit, k group).  grid.x = k-tiles of the longest row block, grid.y =
// row block I - I0.
__global__ __launch_bounds__(256) void pack_oz_kernel(const double *__restrict__ Linv, int64_t ld, int64_t n,
                                                      double sf2, int64_t I0, char *__restrict__ aoz,
                                                      int *__restrict__ eoz) {
    const int64_t I = I0 + blockIdx.y;
    const int64_t kb = blockIdx.x;
    if (kb >= (I + 1) * kTilesPerRowBlockStep) return;
    const int64_t T = tile_start(I) + kb;
    const int rr = threadIdx.x;                 // row within the row block
    const int64_t row = I * kBM + rr;
    double v[kBK];
    double amax = 0.0;
#pragma unroll
    for (int c = 0; c < kBK; ++c) {
        const int64_t col = kb * kBK + c;
        v[c] = (row < n && col < n && col <= row) ? sf2 * Linv[row + col * ld] : 0.0;
        amax = fmax(amax, fabs(v[c]));
    }
    // the 16-row block's max: lanes 16 b .. 16 b + 15 of the wave
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) amax = fmax(amax, __shfl_xor(amax, o));
    int eA = -900;                               // an all-zero block: digits 0, scale negligible
    if (amax > 0.0) {
        int e;
        (void)frexp(amax * 1.01, &e);           // 2^e > 1.01 max |A|: |A| 2^-e < 0.99
        eA = e;
    }
    const int sub = rr >> 4, h = sub >> 3, rb = sub & 7;
    if ((rr & 15) == 0) eoz[T * 16 + sub] = eA;
    char *base = aoz + T * (int64_t)kOzTileBytes + h * kOzA + rb * 1024;
    // XA = rint(A 2^(39 - eA)), |XA| < 2^39 / 1.01, from ONE f64 FMA (round 6;
    // was ldexp + rint + an f64 -> i64 conversion sequence per value, 1.4 ms
    // at C4): fma(A, 2^(39 - eA), 1.5 2^52) is exact up to its one rounding,
    // to the nearest integer with ties to even (the sum lies in [2^52, 2^53):
    // ulp 1; 1.5 2^52 is even), i.e. 1.5 2^52 + rint(A 2^(39 - eA)) -- whose
    // bit pattern is 0x4338000000000000 + XA.  Bitwise the same digits.
    const double scale = eA > -900 ? ldexp(1.0, 39 - eA) : 0.0;   // (all-zero block: XA = 0)
    constexpr double kMagic = 6755399441055744.0;                  // 1.5 2^52
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
        uint32_t w[kOzDigits][4];
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
            // the bytes of XA + 0x80808080 are the digits (the four lower ones + 128)
            const uint64_t yv = (uint64_t)__double_as_longlong(fma(v[16 * gg + jj], scale, kMagic)) -
                                0x4338000000000000ull + 0x80808080ull;
#pragma unroll
            for (int s = 0; s < kOzDigits; ++s) {
                const uint32_t b = (uint32_t)(yv >> (8 * (kOzDigits - 1 - s))) & 0xFFu;
                if ((jj & 3) == 0) w[s][jj >> 2] = b;
                else w[s][jj >> 2] |= b << (8 * (jj & 3));
            }
        }
#pragma unroll
        for (int s = 1; s < kOzDigits; ++s)
#pragma unroll
            for (int q = 0; q < 4; ++q) w[s][q] ^= 0x80808080u;
        const int l = (rr & 15) + 16 * gg;
#pragma unroll
        for (int s = 0; s < kOzDigits; ++s) {
            uint4 *dst = reinterpret_cast<uint4 *>(base + s * kOzPlane + l * 16);
            *dst = make_uint4(w[s][0], w[s][1], w[s][2], w[s][3]);
        }
    }
}

// Per k-tile: x[64], y[64] (f64 of the stored f32), sf2 alpha[64] (f64, alpha
// from the f64 solve), x[64], y[64] (the stored f32, for the sweep's pass-1
// distance); padding rows: the first point's coordinates, alpha 0.
__global__ void pack_koz_kernel(const float *__restrict__ x, const float *__restrict__ y,
                                const double *__restrict__ alpha, int64_t n, int64_t npad, double sf2,
                                char *__restrict__ koz) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= npad) return;
    char *c = koz + (k / kBK) * kOzC;
    const int o = (int)(k % kBK);
    const bool in = k < n;
    reinterpret_cast<double *>(c)[o] = (double)(in ? x[k] : x[0]);
    reinterpret_cast<double *>(c + kBK * 8)[o] = (double)(in ? y[k] : y[0]);
    reinterpret_cast<double *>(c + kBK * 16)[o] = in ? sf2 * alpha[k] : 0.0;
    reinterpret_cast<float *>(c + kBK * 24)[o] = in ? x[k] : x[0];
    reinterpret_cast<float *>(c + kBK * 28)[o] = in ? y[k] : y[0];
}

// ---------------------------------------------------------------------------
// Pair mode (SBO_OPT_PRECISE_KERNEL 4, round 5): A's and
// K*'s exponents shared by a PAIR of k-tiles (2p, 2p + 1), so every level's
// int32 sum chains over 128 k before the f64 combination.  The kernel is
// issue-bound on that combination (profiles/r5_pmc_oz_table.txt: VALU
// instructions 25.8 % of wave cycles against 6.2 % MFMA, matrix pipe 48 %);
// chaining two tiles halves its VALU per MFMA.  Exact integer sums still:
// per level per tile |sum| <= (pairs at the level) 64 2^14, over two tiles
// h23 = l2 256 + l3 + [l4 / 256] < 6 2^28 + 2^23 + 2^15 < 2^31.  The price is
// precision where a pair's two tiles differ in scale (the smaller one keeps
// fewer of its own bits): emulated on the lpsc box at N = 8192
// (tools/r5_emulate_pairs.py, profiles/r5_emulate_pairs.log) the variance
// moves 3.9e-8 -> 6.1e-8 (sn2 0.01: 9.9e-7 -> 1.3e-6; l 0.8: 9.4e-8 -> 1.5e-7).
// Layout: pair (I, p) of a row block = its tiles 2p, 2p + 1 (80 KiB each, the
// same bytes as two kernel-1 tiles) holding four stages of 40 KiB, one per
// quarter of the rows (64 rows = four 16-row blocks): stage piece ((s 2 + e) 4
// + b) = digit s of tile e of block b, 1 KiB in kernel 1's lane order; the
// pair's 16 block exponents at tile 2p's 64 B of eoz.  The K* table per
// (query block, pair): [wave][tile e][digit u][lane][16 B] (64 KiB), eK per
// query (512 B), the pair's mean terms per query (1 KiB).
// Walk: an item's list entries are merged into pairs (entry t and t + 1 for
// t even: one pair; a lone tile of a pair runs with its partner, whose K*
// terms are then included although the plan dropped them -- more work, never
// less accuracy); four stages per pair, double buffered; the pair's table in a
// slot of its own, read into registers at quarter 0 and refilled for the next
// pair at quarter 3.
constexpr int kOz2RB = 4;                                    // 16-row blocks per stage
constexpr int kOz2A = kOzDigits * 2 * kOz2RB * 1024;         // 40 KiB of digits per stage
constexpr int kOz2E = 64;                                    // the pair's 16 block exponents
constexpr int kOz2Slot = kOz2A + kOz2E;
constexpr int kKzt2Digits = kOzWaves * 2 * kOzKDigits * 1024;   // 64 KiB
constexpr int kKzt2E = kKzt2Digits;
constexpr int kKzt2Mu = kKzt2E + kBN * 4;
constexpr int kKzt2 = kKzt2Mu + kBN * 8;                     // 67072 B per (query block, pair)
constexpr int kOz2Smem = 2 * kOz2Slot + kKzt2 + 4096;        // two stage slots, the table, the windows
constexpr int kOz2TableDma = 2 * kOzKDigits + 2;            // DMA instructions per wave per table piece
static_assert(kOz2Smem <= 160 * 1024, "pair-mode LDS");
static_assert(kOz2A == 2 * kOzA / 2 && 4 * kOz2A == 2 * kOzTileBytes, "a pair is two kernel-1 tiles");

// One stage: quarter QQ's four 16-row blocks into this row half's eight
// accumulators (acc[(QQ & 1) 4 + b]), software-pipelined by hand (round 5):
// the stage is eight sub-blocks (block b, tile e), each five digit reads and
// fourteen MFMAs; sub-block i + 1's reads are issued among sub-block i's
// MFMAs, and block b - 1's f64 combination among block b's first sub-block's
// MFMAs (its level sums held in a second register set).  The compiler's own
// schedule issued each sub-block's reads just before their MFMAs and waited
// on them at once (s_waitcnt lgkmcnt(4) right after the reads), and combined
// every block after its last MFMA: the LDS latency and the combination were
// exposed in both waves of a SIMD at the same time.
__device__ __forceinline__ void oz2_read(const i32x4 *__restrict__ pa, int i, i32x4 (&ad)[kOzDigits]) {
    const int b = i >> 1, e = i & 1;
#pragma unroll
    for (int s = 0; s < kOzDigits; ++s) ad[s] = pa[((s * 2 + e) * kOz2RB + b) * 64];
}
struct Oz2Levels {
    i32x4 l0, l1, l2, l3, l4;
};
__device__ __forceinline__ void oz2_products(const i32x4 (&ad)[kOzDigits], const i32x4 (&kd)[kOzKDigits], bool first,
                                             Oz2Levels &L) {
    const i32x4 z = {0, 0, 0, 0}, c128 = {128, 128, 128, 128};
    L.l0 = mfma_i8(ad[0], kd[0], first ? z : L.l0);
    L.l1 = mfma_i8(ad[0], kd[1], first ? z : L.l1);
    L.l2 = mfma_i8(ad[0], kd[2], first ? z : L.l2);
    L.l3 = mfma_i8(ad[0], kd[3], first ? z : L.l3);
    L.l1 = mfma_i8(ad[1], kd[0], L.l1);
    L.l2 = mfma_i8(ad[1], kd[1], L.l2);
    L.l3 = mfma_i8(ad[1], kd[2], L.l3);
    L.l4 = mfma_i8(ad[1], kd[3], first ? c128 : L.l4);
    L.l2 = mfma_i8(ad[2], kd[0], L.l2);
    L.l3 = mfma_i8(ad[2], kd[1], L.l3);
    L.l4 = mfma_i8(ad[2], kd[2], L.l4);
    L.l3 = mfma_i8(ad[3], kd[0], L.l3);
    L.l4 = mfma_i8(ad[3], kd[1], L.l4);
    L.l4 = mfma_i8(ad[4], kd[0], L.l4);
}
__device__ __forceinline__ void oz2_combine(const Oz2Levels &L, double S, f64x4 &acc) {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        const int h01 = L.l0[v] * 256 + L.l1[v];                  // |.| < 2^30
        const int h23 = L.l2[v] * 256 + L.l3[v] + (L.l4[v] >> 8);   // |.| < 2^31 (above)
        const double t = fma((double)h01, 65536.0, (double)h23);
        acc[v] = fma(t, S, acc[v]);
    }
}
// interleave: each of the 14 MFMAs followed by up to three VALU (a pending
// combination)
__device__ __forceinline__ void oz2_interleave(bool combine) {
#pragma unroll
    for (int j = 0; j < 14; ++j) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                  // MFMA
        if (combine) __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);     // VALU
    }
}
template <int QQ>
__device__ __forceinline__ void stage_blocks2(const char *__restrict__ slot, int lane, const i32x4 (&kd)[2][kOzKDigits],
                                              int eK, f64x4 (&acc)[kOzHalfRB]) {
    const int *eA = reinterpret_cast<const int *>(slot + kOz2A);
    const i32x4 *pa = reinterpret_cast<const i32x4 *>(slot) + lane;
    double S[kOz2RB];
#pragma unroll
    for (int b = 0; b < kOz2RB; ++b)
        S[b] = ldexp(1.0, __builtin_amdgcn_readfirstlane(eA[QQ * kOz2RB + b]) + eK - kOzScale);
    i32x4 ad[2][kOzDigits];
    Oz2Levels L[2];
    oz2_read(pa, 0, ad[0]);
#pragma unroll
    for (int i = 0; i < 2 * kOz2RB; ++i) {
        const int b = i >> 1, e = i & 1;
        // the next sub-block's reads stay above this one's MFMAs (a
        // scheduling barrier each side), so their latency hides under them
        if (i + 1 < 2 * kOz2RB) oz2_read(pa, i + 1, ad[(i + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        oz2_products(ad[i & 1], kd[e], e == 0, L[b & 1]);
        const bool comb = e == 0 && b > 0;
        if (comb) oz2_combine(L[(b - 1) & 1], S[b - 1], acc[(QQ & 1) * kOz2RB + b - 1]);
        oz2_interleave(comb);
        __builtin_amdgcn_sched_barrier(0);
    }
    oz2_combine(L[(kOz2RB - 1) & 1], S[kOz2RB - 1], acc[(QQ & 1) * kOz2RB + kOz2RB - 1]);
}

// The sweep walks each item TWICE, once per 128-row half (quarters 0-1, then
// 2-3 of every pair), so that a wave holds eight f64 accumulator blocks, not
// sixteen: with sixteen, the pair's two digit sets and the chained levels
// spilled 72 registers.  The K* table piece is staged once per (pair, half).
// NOTABLE (diagnostic build only, wrong results): the pair tables after the
// first are not staged -- the bound on what the table traffic costs.
template <bool NOTABLE>
__global__ __launch_bounds__(kOzThreads, 1) void predict_oz2_kernel(
    const char *__restrict__ aoz, const int *__restrict__ eoz, const int4 *__restrict__ desc,
    const unsigned short *__restrict__ tl, const int *__restrict__ seg, int P, int n_items, int nI,
    int64_t m, int64_t ldp, double m0, double *__restrict__ part, double *__restrict__ mean,
    const char *__restrict__ kzt) {
    __shared__ __attribute__((aligned(16))) char smem[kOz2Smem];
    const int bid = blockIdx.x;
    const int rng = (P % 8 == 0) ? (bid % 8) * (P / 8) + bid / 8 : bid;
    const int k0 = max(seg[rng], 0), k1 = min(seg[rng + 1], n_items);
    if (k0 >= k1) return;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int r = lane & 15;
    const int g = lane >> 4;
    const int4 *dwin = reinterpret_cast<const int4 *>(smem + 2 * kOz2Slot + kKzt2);
    const unsigned short *lwin = reinterpret_cast<const unsigned short *>(smem + 2 * kOz2Slot + kKzt2 + 2048);
    const char *tz = smem + 2 * kOz2Slot;   // the (pair, half)'s K* table piece

    typedef __attribute__((address_space(3))) char lds_char;
    const uint32_t lds_smem = (uint32_t)(uintptr_t)(lds_char *)(smem);
    const uint32_t lds_wave = lds_smem + (uint32_t)__builtin_amdgcn_readfirstlane(wave) * 1024u;
    const uint32_t lds_tz = lds_smem + 2u * kOz2Slot;
    const uint32_t lds_dwin = lds_tz + (uint32_t)kKzt2;
    const uint32_t lds_lwin = lds_dwin + 2048u;
    const char *gA = aoz + wave * 1024 + lane * 16;
    const char *gE = reinterpret_cast<const char *>(eoz) + lane * 16;
    const char *gD = reinterpret_cast<const char *>(desc) + lane * 16;
    const char *gL = reinterpret_cast<const char *>(tl) + lane * 16;
    const char *gZ = kzt + lane * 16;
    const int wave_u = __builtin_amdgcn_readfirstlane(wave);
    const int npr = kTilesPerRowBlockStep * nI / 2;   // pairs per query block in the table
#define SBO_OZ_DMA16(gsrc, ldst)                                                                         \
    do {                                                                                                 \
        uint32_t keep_;                                                                                  \
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t" \
                     "s_mov_b32 m0, %0"                                                                  \
                     : "=&s"(keep_)                                                                      \
                     : "v"(gsrc), "s"(ldst)                                                              \
                     : "memory");                                                                        \
    } while (0)
    // quarter q_ of pair (first packed tile Tp_) into slot buf
#define SBO_OZ2_STAGE(Tp_, q_, buf)                                                                      \
    do {                                                                                                 \
        const char *s_ = gA + (int64_t)(Tp_) * kOzTileBytes + (q_) * kOz2A;                              \
        const uint32_t d_ = __builtin_amdgcn_readfirstlane(lds_wave + (uint32_t)(buf) * kOz2Slot);       \
        _Pragma("unroll") for (int j_ = 0; j_ < kOz2A / (1024 * kOzWaves); ++j_)                         \
            SBO_OZ_DMA16(s_ + j_ * kOzWaves * 1024, d_ + (uint32_t)(j_ * kOzWaves * 1024));              \
        if (wave == 0 && lane < 4)                                                                       \
            SBO_OZ_DMA16(gE + (int64_t)(Tp_) * 64,                                                       \
                         __builtin_amdgcn_readfirstlane(lds_smem + (uint32_t)((buf) * kOz2Slot + kOz2A)));    \
    } while (0)
    // the table piece of (query block qb_, pair pr_): each wave moves exactly
    // what it reads itself (its digits, its 16 queries' eK and mean terms) --
    // kSbo2TableDma instructions -- so a wave may refill the piece as soon
    // as it has read it, whatever the other waves are doing
#define SBO_OZ2_TABLE(qb_, pr_)                                                                          \
    do {                                                                                                 \
        const char *z_ = gZ + ((int64_t)(qb_) * npr + (pr_)) * kKzt2;                                    \
        _Pragma("unroll") for (int u_ = 0; u_ < 2 * kOzKDigits; ++u_)                                    \
            SBO_OZ_DMA16(z_ + wave * 8192 + u_ * 1024, lds_tz + (uint32_t)(wave_u * 8192 + u_ * 1024));  \
        if (lane < 4) SBO_OZ_DMA16(z_ + kKzt2E + wave * 64, lds_tz + (uint32_t)(kKzt2E + wave_u * 64));  \
        if (lane < 8) SBO_OZ_DMA16(z_ + kKzt2Mu + wave * 128, lds_tz + (uint32_t)(kKzt2Mu + wave_u * 128)); \
    } while (0)
#define SBO_OZ_DESC_WINDOW(w_)                                                                           \
    do {                                                                                                 \
        if (wave == 1) SBO_OZ_DMA16(gD + (int64_t)(w_) * 1024, lds_dwin + (uint32_t)((w_) & 1) * 1024u); \
    } while (0)
#define SBO_OZ_LIST_WINDOW(w_)                                                                           \
    do {                                                                                                 \
        if (wave == 2) SBO_OZ_DMA16(gL + (int64_t)(w_) * 1024, lds_lwin + (uint32_t)((w_) & 1) * 1024u); \
    } while (0)
    auto desc_at = [&](int k) {
        const int4 d = dwin[((k / kOzDescWin) & 1) * kOzDescWin + k % kOzDescWin];
        const int I = min(max(__builtin_amdgcn_readfirstlane(d.x), 0), nI - 1);
        return make_int4(I, __builtin_amdgcn_readfirstlane(d.y), __builtin_amdgcn_readfirstlane(d.z),
                         __builtin_amdgcn_readfirstlane(d.w));
    };
    auto entry_off = [](const int4 &d) {
        return (uint64_t)(uint32_t)d.z | ((uint64_t)((uint32_t)d.w >> 16) << 32);
    };
    auto list_at = [&](uint64_t e, int I) {
        const int t = __builtin_amdgcn_readfirstlane((int)lwin[((e / kOzListWin) & 1) * kOzListWin + e % kOzListWin]) &
                      ((1 << kLevelShift) - 1);
        return min(t, kTilesPerRowBlockStep * (I + 1) - 1);
    };
    // the pair of list entry e (the item's j-th of cnt): its index, and how
    // many entries it takes (2 when entry e + 1 is the partner)
    auto pair_at = [&](uint64_t e, int I, int j, int cnt, int &ne) {
        const int t0 = list_at(e, I);
        ne = 1;
        if ((t0 & 1) == 0 && j + 1 < cnt && list_at(e + 1, I) == t0 + 1) ne = 2;
        return t0 >> 1;
    };

    // ---- prologue
    SBO_OZ_DESC_WINDOW(k0 / kOzDescWin);
    SBO_OZ_DESC_WINDOW(k0 / kOzDescWin + 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int4 dc = desc_at(k0);
    uint64_t e = entry_off(dc);
    SBO_OZ_LIST_WINDOW(e / kOzListWin);
    SBO_OZ_LIST_WINDOW(e / kOzListWin + 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int ne = 1;
    int pr = pair_at(e, dc.x, 0, dc.w & 0xffff, ne);
    int pr0 = pr, ne0 = ne;      // the item's first pair (the second half starts there again)
    SBO_OZ2_STAGE(tile_start(dc.x) + 2 * pr, 0, 0);
    SBO_OZ2_TABLE(dc.y, pr);
    int64_t q = (int64_t)dc.y * kBN + wave * 16 + r;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    f64x4 acc[kOzHalfRB];
#pragma unroll
    for (int rb = 0; rb < kOzHalfRB; ++rb) acc[rb] = f64x4{0.0, 0.0, 0.0, 0.0};
    i32x4 kd[2][kOzKDigits];
    int eK = 0;
    double mu = 0.0, vsum = 0.0;
    // k item, hp row half, j entries of the item before the current pair, sq
    // stage of the pair in this half, cur slot
    int k = k0, hp = 0, j = 0, sq = 0, cur = 0;
    bool table_ahead = false;
    for (;;) {
        const int cnt = dc.w & 0xffff;
        // the next stage: the pair's other quarter of this half, the next pair
        // of this half, the item's first pair again for the second half, or
        // the first pair of item k + 1
        int kn = k, hn = hp, jn = j, sn = sq + 1, prn = pr, nen = ne;
        uint64_t en = e;
        bool restart = false;
        if (sn == 2) {
            sn = 0;
            jn = j + ne;
            en = e + ne;
            if (jn >= cnt) {
                jn = 0;
                if (hp == 0) {
                    hn = 1;
                    en = entry_off(dc);
                    restart = true;
                } else {
                    hn = 0;
                    kn = k + 1;
                }
            }
        }
        const bool more = kn < k1;
        int4 dn = dc;
        if (more) {
            if (kn != k) {
                dn = desc_at(kn);
                if (kn % kOzDescWin == 0) SBO_OZ_DESC_WINDOW(kn / kOzDescWin + 1);
            }
            if (restart) {
                // the item's entries again: its first pair from registers, the
                // list windows reloaded for the pairs after it
                prn = pr0;
                nen = ne0;
                SBO_OZ_LIST_WINDOW(en / kOzListWin);
                SBO_OZ_LIST_WINDOW(en / kOzListWin + 1);
            } else if (sn == 0) {
                if (en / kOzListWin != e / kOzListWin) SBO_OZ_LIST_WINDOW(en / kOzListWin + 1);
                prn = pair_at(en, dn.x, jn, dn.w & 0xffff, nen);
            }
            SBO_OZ2_STAGE(tile_start(dn.x) + 2 * prn, 2 * hn + sn, cur ^ 1);
        }
        const char *slot = smem + cur * kOz2Slot;
        const int I = dc.x;
        const int qq = 2 * hp + sq;
        if (sq == 0) {
#pragma unroll
            for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
                for (int u = 0; u < kOzKDigits; ++u)
                    kd[t2][u] = *reinterpret_cast<const i32x4 *>(tz + wave * 8192 + (t2 * kOzKDigits + u) * 1024 +
                                                                 lane * 16);
            eK = *reinterpret_cast<const int *>(tz + kKzt2E + (wave * 16 + r) * 4);
            if (hp == 0 && I == nI - 1 && g == 0)
                mu += *reinterpret_cast<const double *>(tz + kKzt2Mu + (wave * 16 + r) * 8);
            // the NEXT pair-half's piece, two stages ahead (its latency, not
            // the A stage's, was what the pair sweep waited on: the same sweep
            // without table traffic ran 1538 against 1907 ms,
            // profiles/r5_oz_bounds.log): the next pair of this half, this
            // item's first pair for its second half, or item k + 1's first
            if (!NOTABLE) {
                int qbN = -1, prN = 0, neN = 1;
                if (j + ne < cnt) {
                    prN = pair_at(e + ne, I, j + ne, cnt, neN);
                    qbN = dc.y;
                } else if (hp == 0) {
                    prN = pr0;
                    qbN = dc.y;
                } else if (k + 1 < k1) {
                    const int4 d2 = desc_at(k + 1);
                    prN = pair_at(entry_off(d2), d2.x, 0, d2.w & 0xffff, neN);
                    qbN = d2.y;
                }
                if (qbN >= 0) {
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's reads of the piece are done
                    SBO_OZ2_TABLE(qbN, prN);
                    table_ahead = true;
                }
            }
        }
        if (qq == 0) stage_blocks2<0>(slot, lane, kd, eK, acc);
        else if (qq == 1) stage_blocks2<1>(slot, lane, kd, eK, acc);
        else if (qq == 2) stage_blocks2<2>(slot, lane, kd, eK, acc);
        else stage_blocks2<3>(slot, lane, kd, eK, acc);
        if (sq == 1 && j + ne >= cnt) {
            // the half is done: its rows' V^2 into vsum; after the second
            // half the column sums of the item's 256 rows
#pragma unroll
            for (int rb = 0; rb < kOzHalfRB; ++rb) {
#pragma unroll
                for (int c = 0; c < 4; ++c) vsum = fma(acc[rb][c], acc[rb][c], vsum);
                acc[rb] = f64x4{0.0, 0.0, 0.0, 0.0};
            }
            if (hp == 1) {
                double sum = vsum;
                sum += __shfl_xor(sum, 16);
                sum += __shfl_xor(sum, 32);
                vsum = 0.0;
                const bool writer = lane < 16 && q < m;
                if (writer) part[(int64_t)I * ldp + q] = sum;
                if (I == nI - 1) {
                    mu += __shfl_xor(mu, 16);
                    mu += __shfl_xor(mu, 32);
                    if (writer) mean[q] = m0 + mu;
                    mu = 0.0;
                }
            }
        }
        // the next stage's A must have landed; the table piece issued this
        // step may stay in flight until the end of the next one
        if (table_ahead)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kOz2TableDma) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        table_ahead = false;
        __syncthreads();
        if (!more) break;
        if (kn != k) {
            k = kn;
            dc = dn;
            q = (int64_t)dc.y * kBN + wave * 16 + r;
        }
        if (sn == 0) {
            e = en;
            pr = prn;
            ne = nen;
            if (jn == 0 && hn == 0) {   // a new item: remember its first pair
                pr0 = prn;
                ne0 = nen;
            }
        }
        hp = hn;
        j = jn;
        sq = sn;
        cur ^= 1;
    }
#undef SBO_OZ2_STAGE
#undef SBO_OZ2_TABLE
#undef SBO_OZ_DESC_WINDOW
#undef SBO_OZ_LIST_WINDOW
#undef SBO_OZ_DMA16
}

// The pair-mode K* table (SBO_OPT_PRECISE_KERNEL 4): one workgroup per (pair,
// query block), eK from the smaller distance of the pair's two tiles, then
// each tile's digits under it (kstar_digits' arithmetic), the pair's mean
// terms.  grid = (pairs, query blocks).
__global__ __launch_bounds__(kOzThreads) void kstar_table2_kernel(const char *__restrict__ koz,
                                                                  const float *__restrict__ qx,
                                                                  const float *__restrict__ qy, int64_t m, int npr,
                                                                  int64_t nq, double cexp, char *__restrict__ kzt) {
    __shared__ double T2[64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, r = lane & 15;
    if (tid < 64) T2[tid] = exp2((double)tid * 0.015625);
    __syncthreads();
    const int p = blockIdx.x;
    const char *pc0 = koz + (int64_t)(2 * p) * kOzC, *pc1 = pc0 + kOzC;
    for (int64_t qb = blockIdx.y; qb < nq; qb += gridDim.y) {
        const int64_t q = qb * kBN + wave * 16 + r;
        const double xq = (double)qx[q < m ? q : m - 1], yq = (double)qy[q < m ? q : m - 1];
        const int eK = kstar_exp(fminf(kstar_dmin(pc0, g, xq, yq), kstar_dmin(pc1, g, xq, yq)), cexp);
        char *out = kzt + (qb * npr + p) * (int64_t)kKzt2;
        double mu = 0.0;
#pragma unroll 1
        for (int t2 = 0; t2 < 2; ++t2) {
            i32x4 kd[kOzKDigits];
            kstar_digits_e<true>(t2 ? pc1 : pc0, T2, g, xq, yq, cexp, eK, kd, mu);
#pragma unroll
            for (int u = 0; u < kOzKDigits; ++u)
                *reinterpret_cast<i32x4 *>(out + wave * 8192 + (t2 * kOzKDigits + u) * 1024 + lane * 16) = kd[u];
        }
        mu += __shfl_xor(mu, 16);
        mu += __shfl_xor(mu, 32);
        if (g == 0) {
            reinterpret_cast<int *>(out + kKzt2E)[wave * 16 + r] = eK;
            reinterpret_cast<double *>(out + kKzt2Mu)[wave * 16 + r] = mu;
        }
    }
}

// A = sf2 L^-1 into pair-mode digit tiles for row blocks I >= I0 (the layout
// above): one workgroup per (pair, row block), one thread per row; the 16-row
// block's exponent from the pair's 128 k, then each tile's 64 values as
// pack_oz_kernel cuts them.  grid.x = pairs of the longest row block, grid.y
// = row block I - I0.
__global__ __launch_bounds__(256) void pack_oz2_kernel(const double *__restrict__ Linv, int64_t ld, int64_t n,
                                                       double sf2, int64_t I0, char *__restrict__ aoz,
                                                       int *__restrict__ eoz) {
    const int64_t I = I0 + blockIdx.y;
    const int64_t p = blockIdx.x;
    if (p >= (I + 1) * kTilesPerRowBlockStep / 2) return;
    const int64_t Tp = tile_start(I) + 2 * p;
    const int rr = threadIdx.x;
    const int64_t row = I * kBM + rr;
    auto val = [&](int64_t col) { return (row < n && col < n && col <= row) ? sf2 * Linv[row + col * ld] : 0.0; };
    double amax = 0.0;
    for (int c = 0; c < 2 * kBK; ++c) amax = fmax(amax, fabs(val(p * 2 * kBK + c)));
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) amax = fmax(amax, __shfl_xor(amax, o));
    int eA = -900;
    if (amax > 0.0) {
        int ex;
        (void)frexp(amax * 1.01, &ex);
        eA = ex;
    }
    const int sub = rr >> 4, qq = sub >> 2, b = sub & 3;
    if ((rr & 15) == 0) eoz[Tp * 16 + sub] = eA;
    const double scale = eA > -900 ? ldexp(1.0, 39 - eA) : 0.0;
    char *base = aoz + Tp * (int64_t)kOzTileBytes + qq * kOz2A;
    for (int t2 = 0; t2 < 2; ++t2) {
        double v[kBK];
#pragma unroll
        for (int c = 0; c < kBK; ++c) v[c] = val((2 * p + t2) * kBK + c);
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
            uint32_t w[kOzDigits][4];
#pragma unroll
            for (int jj = 0; jj < 16; ++jj) {
                // (the one-FMA rounding of pack_oz_kernel: bitwise the same digits)
                const uint64_t yv = (uint64_t)__double_as_longlong(fma(v[16 * gg + jj], scale, 6755399441055744.0)) -
                                    0x4338000000000000ull + 0x80808080ull;
#pragma unroll
                for (int s = 0; s < kOzDigits; ++s) {
                    const uint32_t bt = (uint32_t)(yv >> (8 * (kOzDigits - 1 - s))) & 0xFFu;
                    const uint32_t d = s == 0 ? bt : (bt ^ 0x80u);
                    if ((jj & 3) == 0) w[s][jj >> 2] = d;
                    else w[s][jj >> 2] |= d << (8 * (jj & 3));
                }
            }
            const int l = (rr & 15) + 16 * gg;
#pragma unroll
            for (int s = 0; s < kOzDigits; ++s) {
                uint4 *dst = reinterpret_cast<uint4 *>(base + ((s * 2 + t2) * kOz2RB + b) * 1024 + l * 16);
                *dst = make_uint4(w[s][0], w[s][1], w[s][2], w[s][3]);
            }
        }
    }
}

}  // namespace

size_t oz_operand_bytes(int64_t npad) { return (size_t)kOzTileBytes * (size_t)total_tiles(npad / kBM); }
size_t oz_exp_bytes(int64_t npad) { return 64 * (size_t)total_tiles(npad / kBM); }
size_t oz_coord_bytes(int64_t npad) { return (size_t)kOzC * (size_t)(npad / kBK); }

hipError_t launch_pack_oz(hipStream_t s, const double *Linv, int64_t ld, int64_t n, int64_t npad, int64_t I0,
                          double sf2, const float *x, const float *y, const double *alpha, char *aoz, int *eoz,
                          char *koz, bool pairs) {
    const int64_t nI = npad / kBM;
    if (I0 < nI && pairs) {
        hipLaunchKernelGGL(pack_oz2_kernel, dim3((unsigned)(nI * kTilesPerRowBlockStep / 2), (unsigned)(nI - I0)),
                           dim3(256), 0, s, Linv, ld, n, sf2, I0, aoz, eoz);
    } else if (I0 < nI) {
        hipLaunchKernelGGL(pack_oz_kernel, dim3((unsigned)(nI * kTilesPerRowBlockStep), (unsigned)(nI - I0)),
                           dim3(256), 0, s, Linv, ld, n, sf2, I0, aoz, eoz);
    }
    hipLaunchKernelGGL(pack_koz_kernel, dim3((unsigned)((npad + 255) / 256)), dim3(256), 0, s, x, y, alpha, n, npad,
                       sf2, koz);
    return hipGetLastError();
}

hipError_t launch_predict_oz(hipStream_t s, const char *aoz, const int *eoz, const char *koz, const int4 *desc,
                             const unsigned short *tl, const int *seg, int P, int n_items, int nI, const float *qx,
                             const float *qy, int64_t m, int64_t ldp, double ell, double m0, double *part,
                             double *mean, int variant, const char *kzt) {
    if (nI <= 0 || m <= 0) return hipSuccess;
    const double cexp = -1.0 / (2.0 * ell * ell * 0.69314718055994530942);
#ifdef SBO_DIAG
    if (variant == 9) {   // timing bound: no K* digits (wrong results)
        hipLaunchKernelGGL(predict_oz_kernel<1>, dim3((unsigned)P), dim3(kOzThreads), 0, s, aoz, eoz, koz, desc,
                           tl, seg, P, n_items, nI, qx, qy, m, ldp, cexp, m0, part, mean, kzt);
        return hipGetLastError();
    }
#endif
#ifdef SBO_DIAG
    if (variant == 11 || variant == 12) {   // timing bounds: kernel 3 without any stage DMA / the table's
        if (!kzt) return hipErrorInvalidValue;
        if (variant == 11)
            hipLaunchKernelGGL(predict_oz_kernel<3>, dim3((unsigned)P), dim3(kOzThreads), 0, s, aoz, eoz, koz, desc,
                               tl, seg, P, n_items, nI, qx, qy, m, ldp, cexp, m0, part, mean, kzt);
        else
            hipLaunchKernelGGL(predict_oz_kernel<4>, dim3((unsigned)P), dim3(kOzThreads), 0, s, aoz, eoz, koz, desc,
                               tl, seg, P, n_items, nI, qx, qy, m, ldp, cexp, m0, part, mean, kzt);
        return hipGetLastError();
    }
    if (variant == 10) {   // timing bound: pair mode without the table traffic (wrong results)
        hipLaunchKernelGGL(predict_oz2_kernel<true>, dim3((unsigned)P), dim3(kOzThreads), 0, s, aoz, eoz, desc, tl,
                           seg, P, n_items, nI, m, ldp, m0, part, mean, kzt);
        return hipGetLastError();
    }
#endif
    if (variant == 4) {   // pair mode, K*'s digits from the pair table
        if (!kzt) return hipErrorInvalidValue;
        hipLaunchKernelGGL(predict_oz2_kernel<false>, dim3((unsigned)P), dim3(kOzThreads), 0, s, aoz, eoz, desc, tl,
                           seg, P, n_items, nI, m, ldp, m0, part, mean, kzt);
        return hipGetLastError();
    }
#ifdef SBO_DIAG
    if (variant == 5) {   // K*'s digits from the table, A staged a tile ahead
        if (!kzt) return hipErrorInvalidValue;
        hipLaunchKernelGGL(predict_oz3_kernel, dim3((unsigned)P), dim3(kOzThreads), 0, s, aoz, eoz, desc, tl, seg, P,
                           n_items, nI, m, ldp, m0, part, mean, kzt);
        return hipGetLastError();
    }
#endif
    if (variant == 3) {   // K*'s digits from the table
        if (!kzt) return hipErrorInvalidValue;
        hipLaunchKernelGGL(predict_oz_kernel<2>, dim3((unsigned)P), dim3(kOzThreads), 0, s, aoz, eoz, koz, desc,
                           tl, seg, P, n_items, nI, qx, qy, m, ldp, cexp, m0, part, mean, kzt);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(predict_oz_kernel<0>, dim3((unsigned)P), dim3(kOzThreads), 0, s, aoz, eoz, koz, desc, tl,
                       seg, P, n_items, nI, qx, qy, m, ldp, cexp, m0, part, mean, kzt);
    return hipGetLastError();
}

}  // namespace sbo

namespace sbo {
size_t oz_table_bytes(int64_t npad, bool pairs) {   // per query block
    return pairs ? (size_t)kKzt2 * (size_t)(npad / kBK / 2) : (size_t)kKzt * (size_t)(npad / kBK);
}

hipError_t launch_kstar_table(hipStream_t s, const char *koz, const float *qx, const float *qy, int64_t m,
                              int64_t npad, double ell, int64_t nq, char *kzt, bool pairs) {
    if (m <= 0 || nq <= 0) return hipSuccess;
    const double cexp = -1.0 / (2.0 * ell * ell * 0.69314718055994530942);
    const int nkt = (int)(npad / kBK);
    if (pairs) {
        hipLaunchKernelGGL(kstar_table2_kernel, dim3((unsigned)(nkt / 2), (unsigned)std::min<int64_t>(nq, kMaxGridY)),
                           dim3(kOzThreads), 0, s, koz, qx, qy, m, nkt / 2, nq, cexp, kzt);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(kstar_table_kernel, dim3((unsigned)nkt, (unsigned)std::min<int64_t>(nq, kMaxGridY)),
                       dim3(kOzThreads), 0, s, koz, qx, qy, m, nkt, nq, cexp, kzt);
    return hipGetLastError();
}
}  // namespace sbo
