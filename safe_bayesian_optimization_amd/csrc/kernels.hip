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

__global__ void copy_lower_kernel(const float *__restrict__ src, int64_t lds, int64_t n,
                                  float *__restrict__ dst, int64_t ldd) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t j = blockIdx.y;
    if (i < n) dst[i + j * ldd] = i >= j ? src[i + j * lds] : 0.0f;
}

// ------------------------------------------------------------ operand pack
// grid.x = k-tiles of the longest row block, grid.y = row block I.
template <class T>
__global__ __launch_bounds__(256) void pack_operand_kernel(const T *__restrict__ Linv,
                                                           int64_t ld, int64_t n, T sf2,
                                                           float *__restrict__ aug) {
    const int64_t I = blockIdx.y;
    const int64_t kb = blockIdx.x;
    if (kb >= (I + 1) * kTilesPerRowBlockStep) return;
    float *tile = aug + (tile_start(I) + kb) * kTileFloats;
    for (int e = threadIdx.x; e < kTileFloats; e += 256) {
        const int k = e / kBM, r = ((e & 3) << 5) | ((e >> 2) & 31);  // inverse of tile_offset
        const int64_t row = I * kBM + r, col = kb * kBK + k;
        float v = 0.0f;
        if (row < n && col < n && col <= row) v = (float)(sf2 * Linv[row + col * ld]);
        tile[e] = v;
    }
}

__global__ void widen_lower_kernel(const float *__restrict__ src, int64_t lds, int64_t n,
                                   double *__restrict__ dst) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t j = blockIdx.y;
    if (i < n) dst[i + j * n] = i >= j ? (double)src[i + j * lds] : 0.0;
}

__global__ void pack_kcoord_kernel(const float *__restrict__ x, const float *__restrict__ y,
                                   const float *__restrict__ alpha, int64_t n, int64_t npad,
                                   float sf2, float *__restrict__ kcoord) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= npad) return;
    const int64_t t = k / kBK, o = k % kBK;
    float *c = kcoord + t * (3 * kBK);
    const bool in = k < n;
    c[o] = in ? x[k] : x[0];
    c[kBK + o] = in ? y[k] : y[0];
    c[2 * kBK + o] = in ? sf2 * alpha[k] : 0.0f;
}

// Row 1-norms of the packed operand: block I, thread r sums |A[I*BM + r][:]|.
__global__ __launch_bounds__(kBM) void row_l1_kernel(const float *__restrict__ aug, double *__restrict__ row_l1) {
    const int64_t I = blockIdx.x;
    const int r = threadIdx.x;
    const float *t = aug + tile_start(I) * kTileFloats;
    const int64_t nk = (I + 1) * kBM;  // k-tiles 0..2(I+1)-1, each [BK][BM]
    double s = 0.0;
    for (int64_t k = 0; k < nk; ++k) s += fabs((double)t[(k / kBK) * kTileFloats + tile_offset((int)(k % kBK), r)]);
    row_l1[I * kBM + r] = s;
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
// Workgroup (I, qb): rows [I*BM, I*BM+BM) of A = sf2 L^-1 and the BN = 128
// queries [qb*BN, qb*BN+BN).  Wave w owns queries qb*BN + 32w + (l&31) and all
// BM = 128 rows as four 32-row blocks: four accumulators of
// v_mfma_f32_32x32x2_f32 (exact f32, 64 FLOP/clk/SIMD, independent so the
// 64-cycle dependent latency never stalls issue).  The B operand K*[k][q] is
// generated per lane -- lane l holds k = l>>5, q = l&31, exactly the MFMA
// B-fragment map -- so K* never touches LDS or HBM: one exp2 per lane per
// four MFMAs.  The A tile [BK][BM] is staged through LDS (double buffered,
// one barrier per stage); lanes 0-31 / 32-63 read consecutive rows of
// adjacent k (conflict-free).  The mean rides along in the last row block
// (every k visited) as an f64 FMA per k pair.
//
// Exact tile skipping: a k-tile whose bounding box is farther from the
// workgroup's query bounding box than the f32 underflow radius
// (c*d^2 < -160, i.e. |d| > 14.9 l) contributes K* == +0.0 to every product,
// so it adds exactly nothing to any accumulator.  Each workgroup first
// compacts the list of k-tiles it needs (ascending, so the surviving
// accumulation order is unchanged and results are bitwise identical to the
// dense sweep) and only stages and multiplies those.
//
// Accuracy: a single f32 MFMA chain over all N training points accumulates
// ~sqrt(N) roundings on large cancelling terms (2.2e-5 normwise variance
// error at N = 8192, measured on the device and emulated on the host).  The
// chain is therefore cut after every k-tile (BK = 64 k): each tile's MFMA
// chain starts from a zero accumulator and its result is added into an f64
// outer accumulator (2 VALU per accumulator register per tile).
constexpr int kStageFloats = kTileFloats + 3 * kBK;
constexpr int kMaxList = 2048;  // k-tiles a workgroup can list (N <= 131072); beyond: dense
constexpr int kSmemFloats = 2 * kStageFloats + kMaxList + 32;

template <bool MEAN, class OT>
__device__ __forceinline__ void predict_body(const float *__restrict__ tiles,
                                             const float *__restrict__ kc, const int *tlist,
                                             int cnt, float xq, float yq, float cexp, float *smem,
                                             OT (&outer)[4][16], double &mu) {
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int half = lane >> 5;
    const int row = lane & 31;

    // LDS-DMA staging (global_load_lds_dwordx4): each wave instruction moves
    // 1 KiB, lane-linear; no staging registers.  A stage = the 32 KiB [BK][BM]
    // tile (8 instructions per wave) + 768 B of per-k coordinates (wave 0,
    // lanes 0-47).
    const int wave = tid >> 6;
    typedef __attribute__((address_space(3))) void lds_void;
    const char *gA = reinterpret_cast<const char *>(tiles) + wave * 1024 + lane * 16;
    const char *gC = reinterpret_cast<const char *>(kc) + lane * 16;
    char *lA = reinterpret_cast<char *>(smem) + wave * 1024;
    constexpr int kTileBytes = kTileFloats * 4, kStageBytes = kStageFloats * 4, kCBytes = 3 * kBK * 4;
#define SBO_STAGE(kb, buf)                                                                          \
    do {                                                                                            \
        const char *s_ = gA + (int64_t)(kb) * kTileBytes;                                           \
        char *d_ = lA + (buf) * kStageBytes;                                                        \
        _Pragma("unroll") for (int j = 0; j < kTileBytes / 4096; ++j)                               \
            __builtin_amdgcn_global_load_lds((const void *)(s_ + j * 4096), (lds_void *)(d_ + j * 4096), \
                                             16, 0, 0);                                             \
        if (wave == 0 && lane < kCBytes / 16)                                                       \
            __builtin_amdgcn_global_load_lds((const void *)(gC + (int64_t)(kb) * kCBytes),          \
                                             (lds_void *)(reinterpret_cast<char *>(smem) +          \
                                                          (buf) * kStageBytes + kTileBytes),        \
                                             16, 0, 0);                                             \
    } while (0)

    f32x16 acc[4];
    const f32x16 zero = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (cnt == 0) return;

    SBO_STAGE(tlist ? tlist[0] : 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = 0; i < cnt; ++i) {
        const int cur = i & 1;
        if (i + 1 < cnt) SBO_STAGE(tlist ? tlist[i + 1] : i + 1, cur ^ 1);
        // per-lane bases; every k step is a constant offset from them (LDS
        // immediate offsets, no per-step address registers)
        const float4 *pa = reinterpret_cast<const float4 *>(smem + cur * kStageFloats) + half * 32 + row;
        const float *pc = smem + cur * kStageFloats + kTileFloats + half;
        // software pipeline: the A operands (one ds_read_b128 = the four row
        // blocks, tile_offset layout) and K* of k step p+1 are fetched and
        // evaluated while the four MFMAs of step p run
        float4 a_cur = pa[0];
        float b_cur;
        {
            const float dx = pc[0] - xq, dy = pc[kBK] - yq;
            b_cur = fast_exp2(cexp * fmaf(dy, dy, dx * dx));
        }
#pragma unroll
        for (int p = 0; p < kBK / 2; ++p) {
            float4 a_nxt = a_cur;
            float b_nxt = b_cur;
            if (p + 1 < kBK / 2) {
                a_nxt = pa[(p + 1) * 64];
                const float dx = pc[2 * (p + 1)] - xq, dy = pc[kBK + 2 * (p + 1)] - yq;
                b_nxt = fast_exp2(cexp * fmaf(dy, dy, dx * dx));
            }
            if (MEAN) mu = fma((double)pc[2 * kBK + 2 * p], (double)b_cur, mu);
            acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a_cur.x, b_cur, p == 0 ? zero : acc[0], 0, 0, 0);
            acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a_cur.y, b_cur, p == 0 ? zero : acc[1], 0, 0, 0);
            acc[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a_cur.z, b_cur, p == 0 ? zero : acc[2], 0, 0, 0);
            acc[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(a_cur.w, b_cur, p == 0 ? zero : acc[3], 0, 0, 0);
            a_cur = a_nxt;
            b_cur = b_nxt;
        }
#pragma unroll
        for (int rb = 0; rb < 4; ++rb)
#pragma unroll
            for (int r = 0; r < 16; ++r) outer[rb][r] += (OT)acc[rb][r];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
#undef SBO_STAGE
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

// OT: outer (cross-tile) accumulator type; W: waves per SIMD the register
// budget is fitted to (f64 outer needs 2; f32 outer can run 3).
template <class OT, int W>
__global__ __launch_bounds__(256, W) void predict_kernel(const float *__restrict__ aug,
                                                         const float *__restrict__ kcoord,
                                                         const float4 *__restrict__ kbox, int nI,
                                                         int nQ, const float *__restrict__ qx,
                                                         const float *__restrict__ qy, int64_t m,
                                                         int64_t ldp, float cexp, float skip_d2,
                                                         float m0, float *__restrict__ part,
                                                         float *__restrict__ mean,
                                                         unsigned long long *__restrict__ tiles_done) {
    __shared__ __attribute__((aligned(16))) float smem[kSmemFloats];
    int *tlist = reinterpret_cast<int *>(smem + 2 * kStageFloats);
    float *wbox = smem + 2 * kStageFloats + kMaxList;       // [4 waves][4]
    int *wcnt = reinterpret_cast<int *>(wbox + 16);         // [4 waves]
    const int64_t bid = blockIdx.x;
    const int I = nI - 1 - (int)(bid / nQ);  // heaviest row blocks first
    const int64_t qb = bid % nQ;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int nkb = (I + 1) * kTilesPerRowBlockStep;
    const float *tiles = aug + tile_start(I) * kTileFloats;

    const int64_t q = qb * kBN + wave * 32 + (lane & 31);
    const int64_t qc = q < m ? q : m - 1;
    const float xq = qx[qc], yq = qy[qc];

    // ---- list the k-tiles this workgroup needs (ascending)
    int cnt = nkb;
    const int *list = nullptr;
    if (skip_d2 > 0.0f && nkb <= kMaxList) {
        const float bx0 = wave_min(xq), bx1 = wave_max(xq), by0 = wave_min(yq), by1 = wave_max(yq);
        if (lane == 0) {
            wbox[wave * 4 + 0] = bx0; wbox[wave * 4 + 1] = bx1;
            wbox[wave * 4 + 2] = by0; wbox[wave * 4 + 3] = by1;
        }
        __syncthreads();
        float qx0 = wbox[0], qx1 = wbox[1], qy0 = wbox[2], qy1 = wbox[3];
#pragma unroll
        for (int w = 1; w < 4; ++w) {
            qx0 = fminf(qx0, wbox[w * 4 + 0]); qx1 = fmaxf(qx1, wbox[w * 4 + 1]);
            qy0 = fminf(qy0, wbox[w * 4 + 2]); qy1 = fmaxf(qy1, wbox[w * 4 + 3]);
        }
        int base = 0;
        for (int t0 = 0; t0 < nkb; t0 += 256) {
            const int t = t0 + tid;
            bool keep = false;
            if (t < nkb) {
                const float4 b = kbox[t];  // (xmin, xmax, ymin, ymax); empty tile = (+inf, -inf, ..)
                const float dx = fmaxf(0.0f, fmaxf(b.x - qx1, qx0 - b.y));
                const float dy = fmaxf(0.0f, fmaxf(b.z - qy1, qy0 - b.w));
                keep = fmaf(dy, dy, dx * dx) <= skip_d2;
            }
            const unsigned long long bal = __ballot(keep);
            const int before = __popcll(bal & ((1ull << lane) - 1ull));
            __syncthreads();  // previous chunk's wcnt reads are done
            if (lane == 0) wcnt[wave] = __popcll(bal);
            __syncthreads();
            int off = base;
            for (int w = 0; w < wave; ++w) off += wcnt[w];
            if (keep) tlist[off + before] = t;
            base += wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
        }
        __syncthreads();
        cnt = base;
        list = tlist;
    }
    if (tid == 0 && tiles_done) atomicAdd(tiles_done, (unsigned long long)cnt);  // executed-work counter

    OT outer[4][16];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int r = 0; r < 16; ++r) outer[rb][r] = (OT)0;
    double mu = 0.0;

    const bool last = (I == nI - 1);
    if (last)
        predict_body<true, OT>(tiles, kcoord, list, cnt, xq, yq, cexp, smem, outer, mu);
    else
        predict_body<false, OT>(tiles, kcoord, list, cnt, xq, yq, cexp, smem, outer, mu);

    // epilogue: column sums of V^2 over this block's rows; lanes l and l+32 hold
    // the two row halves of column l&31 of each 32x32 accumulator
    double s = 0.0;
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int r = 0; r < 16; ++r) s = fma((double)outer[rb][r], (double)outer[rb][r], s);
    s += __shfl_xor(s, 32);
    mu += __shfl_xor(mu, 32);
    if (lane < 32 && q < m) {
        part[(int64_t)I * ldp + q] = (float)s;
        if (last) mean[q] = (float)((double)m0 + mu);
    }
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
__device__ __forceinline__ void compute_sets_one(float mu, float sd, double beta, double f_min,
                                                 double &lo, double &hi, bool &safe) {
    const double c = __dmul_rn(beta, (double)sd);
    lo = __dsub_rn((double)mu, c);
    hi = __dadd_rn((double)mu, c);
    safe = lo > f_min;
}

__global__ __launch_bounds__(kAcqThreads) void acquire_kernel(
    const float *__restrict__ part, const float *__restrict__ mean, int nI, int64_t ldp, int64_t m,
    float sf2, double beta, double f_min, int score_kind, int64_t index_offset,
    const int32_t *__restrict__ perm, float *__restrict__ mu_out, float *__restrict__ sd_out,
    double *__restrict__ lo_out, double *__restrict__ hi_out, uint8_t *__restrict__ safe_out,
    sbo_key *__restrict__ keys) {
    const int64_t i = (int64_t)blockIdx.x * kAcqThreads + threadIdx.x;
    double bs = 0.0;
    int64_t bi = -1;
    if (i < m) {
        double s = 0.0;
        for (int I = 0; I < nI; ++I) s += (double)part[(int64_t)I * ldp + i];
        double vd = (double)sf2 - s;
        float var = vd > 0.0 ? (float)vd : 0.0f;
        const float sd = __fsqrt_rn(var);
        const float mu = mean[i];
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

__global__ __launch_bounds__(kAcqThreads) void sets_kernel(const float *__restrict__ mu,
                                                           const float *__restrict__ sd, int64_t m,
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
    hipLaunchKernelGGL(copy_lower_kernel, dim3((unsigned)((n + 255) / 256), (unsigned)n), dim3(256), 0, s,
                       src, ld_src, n, dst, ld_dst);
    return hipGetLastError();
}

template <class T>
hipError_t launch_pack_operand_t(hipStream_t s, const T *Linv, int64_t ld, int64_t n, int64_t npad, double sf2,
                                 const float *x, const float *y, const float *alpha, float *aug, float *kcoord) {
    const int64_t nI = npad / kBM;
    hipLaunchKernelGGL(pack_operand_kernel<T>, dim3((unsigned)(nI * kTilesPerRowBlockStep), (unsigned)nI),
                       dim3(256), 0, s, Linv, ld, n, (T)sf2, aug);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(pack_kcoord_kernel, dim3((unsigned)((npad + 255) / 256)), dim3(256), 0, s, x, y,
                       alpha, n, npad, (float)sf2, kcoord);
    return hipGetLastError();
}

hipError_t launch_pack_operand(hipStream_t s, const float *Linv, int64_t ld, int64_t n, int64_t npad, double sf2,
                               const float *x, const float *y, const float *alpha, float *aug, float *kcoord) {
    return launch_pack_operand_t<float>(s, Linv, ld, n, npad, sf2, x, y, alpha, aug, kcoord);
}

hipError_t launch_pack_operand(hipStream_t s, const double *Linv, int64_t ld, int64_t n, int64_t npad, double sf2,
                               const float *x, const float *y, const float *alpha, float *aug, float *kcoord) {
    return launch_pack_operand_t<double>(s, Linv, ld, n, npad, sf2, x, y, alpha, aug, kcoord);
}

hipError_t launch_widen_lower(hipStream_t s, const float *src, int64_t ld_src, int64_t n, double *dst) {
    hipLaunchKernelGGL(widen_lower_kernel, dim3((unsigned)((n + 255) / 256), (unsigned)n), dim3(256), 0, s, src,
                       ld_src, n, dst);
    return hipGetLastError();
}

hipError_t launch_row_l1(hipStream_t s, const float *aug, int64_t npad, double *row_l1) {
    hipLaunchKernelGGL(row_l1_kernel, dim3((unsigned)(npad / kBM)), dim3(kBM), 0, s, aug, row_l1);
    return hipGetLastError();
}

hipError_t launch_tile_boxes(hipStream_t s, const float *x, const float *y, int64_t n, int64_t npad, float4 *kbox) {
    const int64_t nt = npad / kBK;
    hipLaunchKernelGGL(tile_box_kernel, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, s, x, y, n, nt, kbox);
    return hipGetLastError();
}

hipError_t launch_predict(hipStream_t s, const float *aug, const float *kcoord, const float4 *kbox, int64_t npad,
                          const float *qx, const float *qy, int64_t m, int64_t ldp, float ell, float m0, int skip_log2,
                          float *part, float *mean, unsigned long long *tiles_done, int variant) {
    const int nI = (int)(npad / kBM);
    const int64_t nQ = (m + kBN - 1) / kBN;
    const double ce = -1.0 / (2.0 * (double)ell * (double)ell * 0.69314718055994530942);
    const float cexp = (float)ce;
    // k-tiles farther than this squared distance give c*d^2 < -skip_log2, i.e.
    // every K* entry < 2^-skip_log2 (0.1% margin over the kernel's rounding);
    // skip_log2 >= 150 means every such entry is exactly +0.0 in f32
    const float skip_d2 = skip_log2 > 0 ? (float)((double)skip_log2 / -ce * 1.001) : -1.0f;
    const int64_t blocks = (int64_t)nI * nQ;
    if (blocks > 0x7fffffff) return hipErrorInvalidValue;
#define SBO_PREDICT_ARGS aug, kcoord, kbox, nI, (int)nQ, qx, qy, m, ldp, cexp, skip_d2, m0, part, mean, tiles_done
    switch (variant) {
        case 1: hipLaunchKernelGGL((predict_kernel<float, 2>), dim3((unsigned)blocks), dim3(256), 0, s, SBO_PREDICT_ARGS); break;
        case 2: hipLaunchKernelGGL((predict_kernel<float, 3>), dim3((unsigned)blocks), dim3(256), 0, s, SBO_PREDICT_ARGS); break;
        default: hipLaunchKernelGGL((predict_kernel<double, 2>), dim3((unsigned)blocks), dim3(256), 0, s, SBO_PREDICT_ARGS); break;
    }
#undef SBO_PREDICT_ARGS
    return hipGetLastError();
}

hipError_t launch_acquire(hipStream_t s, const float *part, const float *mean, int nI, int64_t ldp,
                          int64_t m, float sf2, double beta, double f_min, int score_kind,
                          int64_t index_offset, const int32_t *perm, float *mu, float *sd, double *lo,
                          double *hi, uint8_t *safe, sbo_key *block_keys) {
    hipLaunchKernelGGL(acquire_kernel, dim3((unsigned)acq_blocks(m)), dim3(kAcqThreads), 0, s, part, mean,
                       nI, ldp, m, sf2, beta, f_min, score_kind, index_offset, perm, mu, sd, lo, hi, safe,
                       block_keys);
    return hipGetLastError();
}

hipError_t launch_sets(hipStream_t s, const float *mu, const float *sd, int64_t m, double beta,
                       double f_min, double *lo, double *hi, uint8_t *safe) {
    hipLaunchKernelGGL(sets_kernel, dim3((unsigned)acq_blocks(m)), dim3(kAcqThreads), 0, s, mu, sd, m, beta,
                       f_min, lo, hi, safe);
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
