// sbo_internal.hpp -- context state, device buffers and kernel launchers of
// libsbo.so.  Not part of the public ABI (include/sbo.h is).
#pragma once

#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <cstddef>
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "../../include/sbo.h"

namespace sbo {

// ---------------------------------------------------------------- geometry
// Predictive operand tiling (see DESIGN.md "predictive sweep").
//   BM rows of A = sf2 * L^-1 per workgroup, BN queries per workgroup
//   (8 waves x 16), BK training points per LDS stage.
constexpr int kBM = 256;
constexpr int kBN = 128;
constexpr int kBK = 64;
constexpr int kTileFloats = kBM * kBK;           // one packed [BK][BM] tile
constexpr int kTilesPerRowBlockStep = kBM / kBK;  // k-tiles added per row block
constexpr int kAcqThreads = 256;
// grid.y / grid.z of a launch stay below the device limit (65535 on gfx950);
// kernels that index columns by blockIdx.y loop over j += gridDim.y
constexpr int64_t kMaxGridY = 65535;

__host__ __device__ inline int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

// First packed tile of row block I: sum_{I'<I} (I'+1)*(BM/BK).
__host__ __device__ inline int64_t tile_start(int64_t I) { return kTilesPerRowBlockStep * I * (I + 1) / 2; }
inline int64_t total_tiles(int64_t nI) { return tile_start(nI); }
// raster-grid query blocks (query_order.hip): kGridPatchFast points along
// the grid's fast axis x kGridPatchSlow rows
constexpr int kGridPatchFast = 8, kGridPatchSlow = 16;
static_assert(kGridPatchFast * kGridPatchSlow == kBN, "a grid patch is one query block");
struct QueryGrid {
    bool ok = false;
    int64_t W = 0, c0 = 0, R = 0, npf = 0, ms = 0;  // row length, first row's column, rows, patches per row, positions
    int64_t nfull = 0, wl = 0;  // whole patch rows; the last rows' patch width (kBN / the next power of two >= R % 16)
};
inline int64_t grid_max_positions(int64_t m) { return round_up(m + m / 8 + kBN, kBN); }
// Element offset inside a packed [BK][BM] tile of A[row][k] (row < BM, k < BK).
// The MFMA is 16x16x4: lane (k&3, row&15) of a k step needs A of the sixteen
// 16-row blocks of its row; blocks 4jj..4jj+3 sit side by side, so four
// conflict-free ds_read_b128 per lane fetch the A operands of all sixteen
// MFMAs of a step.
__host__ __device__ constexpr int tile_offset(int k, int row) {
    return (((row >> 6) * kBK + k) * 16 + (row & 15)) * 4 + ((row >> 4) & 3);
}

// ----------------------------------------------------------- device buffer
class DevBuf {
public:
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() { release(); }
    // Grow-only; contents are NOT preserved on growth.
    hipError_t reserve(size_t bytes) {
        if (bytes <= cap_) return hipSuccess;
        release();
        hipError_t e = hipMalloc(&ptr_, bytes);
        if (e != hipSuccess) { ptr_ = nullptr; return e; }
        cap_ = bytes;
        return hipSuccess;
    }
    void release() {
        if (ptr_) (void)hipFree(ptr_);
        ptr_ = nullptr;
        cap_ = 0;
    }
    template <class T> T *as() const { return static_cast<T *>(ptr_); }
    void swap(DevBuf &o) {
        std::swap(ptr_, o.ptr_);
        std::swap(cap_, o.cap_);
    }
    size_t capacity() const { return cap_; }

private:
    void *ptr_ = nullptr;
    size_t cap_ = 0;
};

}  // namespace sbo

struct sbo_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    rocblas_handle blas = nullptr;
    // the blocked Cholesky's look-ahead: trailing updates on a second stream
    // (created on first use), ordered against `stream` by two events, with a
    // rocBLAS handle of its own (a handle's device workspace must not be
    // shared by kernels in flight on two streams)
    hipStream_t aux_stream = nullptr;
    rocblas_handle blas_aux = nullptr;
    int chol_reserve = 0;        // SBO_OPT_CHOL_RESERVE: CUs the trailing updates leave free (CU-masked aux stream)
    int aux_reserved = 0;        // the mask the current aux stream was created with
    hipEvent_t ev_panel = nullptr, ev_trail = nullptr;
    hipEvent_t ev_pack = nullptr;  // the fit's operand packs on aux_stream (refresh_operand)
    // the precise operand's pack, left running on aux_stream after the fit's
    // host sync (round 6): the precise sweep waits on it on the device, and
    // anything that rewrites L^-1, alpha64 or the operand first on the host
    hipEvent_t ev_poz = nullptr;
    bool poz_pending = false;
    int chol_gemm_own = 4;       // SBO_OPT_CHOL_GEMM: 4 (default) / 5 the outer panels' updates int8-sliced, 3 split bf16, 2 every update by chol_update_kernel, 1 the small trailing ones, 0 rocBLAS
    int chol_diag = 1;           // SBO_OPT_CHOL_DIAG: 1 the MFMA chain kernels (diagonal block, panel), 0 the VALU ones (bitwise equal)
    int chol_outer = 1024;       // SBO_OPT_CHOL_OUTER: outer panel width of the two-level Cholesky (128: one level)
    // the recursive inverse's first half beside the Cholesky's last steps
    // (SBO_OPT_INV_OVERLAP = R > 0: on inv_stream, CU-masked to leave R CUs free)
    hipStream_t inv_stream = nullptr;
    rocblas_handle blas_inv = nullptr;
    int inv_overlap = 0, inv_reserved = 0;
    hipEvent_t ev_half = nullptr, ev_inv = nullptr;
    int64_t inv_base = 2048;     // SBO_OPT_INV_BASE: dtrtri base case of the recursive inverse
    int64_t inv_panels = 16;     // SBO_OPT_INV_PANELS: dgemm panels per product of the recursion
    int inv_oz = 6;              // SBO_OPT_INV_OZ: digits of the int8-sliced top-level products (0: dgemm)
    int64_t inv_oz_min = 0;      // SBO_OPT_INV_OZ_MIN: the smallest sliced split (0: 2048 at N >= 12288, else 4096)
    bool inv_oz_off = false;     // (set while a fit redoes its inverse with dgemm products: the guard fired)
    // SBO_OPT_INV_OZ_ADAPT: the digits of the current fit's sliced products
    // (inv_digits), those the last guard reading allows for the next fit of
    // the same hyper-parameters, about the same N and box area (0: inv_oz), that
    // reading's N and hyper-parameters, and whether a reduced fit of this data
    // fired (then it keeps inv_oz digits)
    int inv_oz_adapt = 1;
    int inv_oz_cur = 0, inv_oz_next = 0;
    int64_t inv_oz_hist_n = 0;
    double inv_oz_hist_area = 0.0;   // (the training bounding box's area: N / area the density)
    sbo_hyper inv_oz_hist_hyper{};
    bool inv_oz_pinned = false;
    // the inverse's accuracy guard (SBO_OPT_INV_CHECK, inv_check.hip): its
    // stream, workspace, timing events and the last result
    int inv_check = 1;           // SBO_OPT_INV_CHECK: 0 off, 1 after sliced inverses, 2 after every full inverse
    hipStream_t chk_stream = nullptr;
    hipEvent_t ev_chk0 = nullptr, ev_chk1 = nullptr;
    sbo::DevBuf chk;
    sbo_inv_check chk_res{};     // (ran = 0: none since the last fit)
    int64_t early_inv_n = 0;     // n of a factor whose inverse's first half is done (refresh_operand finishes it)
    int inv_slot = 0;            // info slots the first half used (1 .. inv_slot)
    std::string err;

    // fitted model
    int64_t n = 0;       // training points
    int64_t cap = 0;     // allocated leading dimension of L (>= n, for appends)
    sbo_hyper hyper{0.4, 1.0, 0.1, 0.0};
    bool fitted = false;
    bool has_factor = false;     // false after sbo_import_state: predict-only (no L to append to)

    sbo::DevBuf x, y, obs;       // training data, f32, capacity cap
    sbo::DevBuf L;               // lower Cholesky factor, column-major, lda = cap
    sbo::DevBuf Linv;            // L^-1 (strtri f32 workspace, or dtrtri f64 kept for appends), lda = cap
    int64_t linv_n = 0;          // rows of the f64 L^-1 held in Linv (0: none; appends extend it)
    int inverse_bits = 64;       // SBO_OPT_INVERSE_BITS: precision of the L^-1 computation
    int jitter_retries = 0;      // SBO_OPT_JITTER_RETRIES: NOT_SPD fits retried with diagonal jitter
    double jitter = 0.0;         // the diagonal jitter of the current fit (0 unless a retry succeeded)
    bool inverse_rec = true;     // SBO_OPT_INVERSE: 1 own recursive f64 inverse (panelled dgemms), 0 rocSOLVER dtrtri
    bool chol_blocked = true;    // SBO_OPT_CHOLESKY: 1 own blocked factorization, 0 rocSOLVER spotrf
    bool chol_trsm_own = true;   //   1: its panels by chol_trsm_kernel, 2: by rocBLAS strsm
    int spatial_order = 3;       // SBO_OPT_SPATIAL_ORDER: 0 caller order, 1 Hilbert, 2 Morton, 3 k-d
    int skip_log2 = -1;          // SBO_OPT_TILE_SKIP: skip K* tiles with every entry < 2^-L (-1: auto)
    int auto_skip_log2 = 160;    // auto K* cutoff for V (half the budget), computed at fit (refresh_operand)
    int auto_skip_mean_log2 = 160;  // auto cutoff the last row block keeps for the mean
    float lg_tau_v = -1000.0f;   // log2 of each row block's |dV_I|_2 budget (tile-norm test)
    sbo::DevBuf tile_lgn;        // per packed tile: log2 gain bounds of A_It and of its bf16 pieces (2 x float4)
    int skip_budget = 20;        // SBO_OPT_SKIP_BUDGET: the auto cutoff keeps the skip error below 2^-B
    double max_row_l1 = 0.0;     // max_i sum_j |A_ij|, A = sf2 L^-1
    double alpha_l1 = 0.0;       // sum_j |sf2 alpha_j|
    std::vector<int64_t> order;  // internal row -> caller's training index
    float bbox[4] = {0.f, 0.f, 0.f, 0.f};  // training bounding box (x0, x1, y0, y1)
    int query_order = 1;         // SBO_OPT_QUERY_ORDER: 0 caller order, 1 grid patches or Morton, 2 Morton
    // grid layout of the last query buffers seen (the layout depends on (m, W, c0) only)
    const float *qgrid_x = nullptr, *qgrid_y = nullptr;
    int64_t qgrid_m = -1;
    sbo::QueryGrid qgrid;
    sbo::DevBuf qgwork;          // grid detection + patch layout workspace
    int kernel_variant = 3;      // SBO_OPT_KERNEL_VARIANT: predictive kernel (3: split-operand bf16 sweep)
    int sweep_groups = 0;        // SBO_OPT_SWEEP_GROUPS: persistent sweep workgroups (0: one per CU)
    int num_cu = 0;              // compute units of the device
    sbo::DevBuf plan_work;       // the tick's tile plan (launch_plan)
    sbo::DevBuf fwork, fowner, fimg, fpix, fout;  // device frontier (sbo_frontier / sbo_subgoal)
    sbo::DevBuf qwork;           // query ordering workspace
    // the probe's second sweep reads the same queries: reuse the first's
    // Morton order (pointers into qwork; valid only while reuse_order is set)
    bool reuse_order = false;
    int32_t *order_p = nullptr;
    float *order_sx = nullptr, *order_sy = nullptr;
    sbo::DevBuf kbox;            // per k-tile bounding boxes (float4)
    sbo::DevBuf alpha;           // K^-1 (y - m0), length cap
    sbo::DevBuf aug;             // packed sf2 * L^-1 tiles
    sbo::DevBuf kcoord;          // per k-tile: x[BK], y[BK], sf2*alpha[BK]
    sbo::DevBuf ax3, kc3;        // split (bf16 x3) operand and its coordinates (kernel variants 2, 3)
    int64_t x3_I0 = 0;           // first row block whose split operand is stale (>= nI: current)
    int x3_layout = -1;          // layout of the derived split operand (sbo::x3_layout)
    sbo::DevBuf qpad;            // queries padded to whole blocks (split sweep without query ordering)
    sbo::DevBuf qcost;           // sbo_query_cost scratch
    sbo::DevBuf info;            // rocSOLVER info
    sbo::DevBuf scratch;         // append workspace
    int64_t npad = 0;            // rows/cols of the packed operand (multiple of BM)
    // precise sweep (SBO_OPT_PRECISION, predict_f64.hip)
    int precision_opt = -1;      // -1 auto (fit-time probe), 0 the fast split sweep, 1 always f64
    int resort_pct = 25;         // SBO_OPT_RESORT: re-sort + refactor on append past this share of unsorted points
    int64_t n_sorted = 0;        // points of the last k-d sort (fit / re-sort)
    sbo::DevBuf restage;         // the re-sort's staging copy of all points
    bool precise = false;        // the sweep ticks run in effect
    sbo::DevBuf alpha64;         // alpha from the f64 solve (length cap)
    sbo::DevBuf zvec, rvec;      // z = L^-1 (y - m0) (f64, valid for z_n points: appends update alpha from it), r scratch
    sbo::DevBuf awork;           // launch_alpha_f64's partial sums
    int64_t z_n = 0;
    sbo::DevBuf a64, kc64;       // f64 packed operand and coordinates, derived lazily
    sbo::DevBuf aoz, eoz, koz;   // int8 digit operand, its block exponents, coordinates (predict_oz.hip)
    sbo::DevBuf gzws;            // the int8-sliced GEMM's packed operands (SBO_OPT_INV_OZ)
    sbo::DevBuf gzws_aux;        //   and those of the products on aux_stream (the inverse's second half)
    sbo::DevBuf cholx3[2];       // the Cholesky's outer panels split into bf16 planes (SBO_OPT_CHOL_GEMM 3), alternating
    sbo::DevBuf kzt;             // the int8 sweep's K* table of one chunk of query blocks (SBO_OPT_PRECISE_KERNEL 3)
    int precise_kernel = 3;      // SBO_OPT_PRECISE_KERNEL: 0 the f64 MFMA sweep, 1 the int8 sliced sweep, 3 the same reading the K* table
    int64_t a64_I0 = 0;          // first row block whose precise operand (of precise_kernel) is stale
    int64_t probe_n = 0;         // training points at the last probe (0: none)
    double probe_err = -1.0, probe_vmin = 0.0, probe_vmax = 0.0;  // fast sweep's error on the probe, var range
    // the probe's two parts: its grid over the training box, and training
    // locations (where the variance is smallest); each part's own normwise error
    double probe_err_grid = -1.0, probe_err_train = -1.0, probe_vmax_grid = 0.0, probe_vmax_train = 0.0;
    int probe_m_grid = 0, probe_m_train = 0;
    int64_t table_mb = 0;        // SBO_OPT_TABLE_MB: the K* table's memory budget (SBO_OPT_PRECISE_KERNEL 3; 0: auto)
    int probe_grid = 32, probe_train = 512;  // SBO_OPT_PROBE_SIZE: the probe's grid side and training locations
    int plan_block = 0;          // SBO_OPT_PLAN_BLOCK: the precise plans' item blocks (bi << 8 | bq; 0: row-block-major)
    int reprobe_pct = 25;        // SBO_OPT_REPROBE: appends re-probe once N grew by this share (0: every append)
    bool inv_batched = true;      // SBO_OPT_INV_LEAVES: the recursion's base cases inverted up front, batched
    bool inv_leaves_own = true;   // (SBO_OPT_INV_LEAVES 2, default: by doubling from 128-column blocks, inverse_leaves)
    bool inv_leaves_done = false; // (set while a recursion runs whose base cases are already inverted)
    int64_t widened_n = 0;       // blocked_potrf widened the factor into Linv (n) for refresh_operand
    double probe_ref_tol = 0.0;  // the probe reference sweep's skip budget (absolute variance)
    int p_skip_log2 = 160;       // the precise plan's cutoffs and budget (2^-B of the probe's smallest variance)
    float p_lg_tau_v = -1000.0f;
    sbo::DevBuf qprobe, oprobe;  // probe grid and outputs

    // per-call staging
    sbo::DevBuf part, mean;      // predictive partial sums [nI][ldp], mean [ldp]
    sbo::DevBuf hq;              // host-input staging (queries, mu/sd, ...)
    sbo::DevBuf hout;            // host-output staging
    sbo::DevBuf keys;            // per-block argmax keys + final key
    sbo_key *host_key = nullptr; // pinned readback

    // kernel timing (sbo_profile)
    bool prof = false;
    std::vector<hipEvent_t> ev_pool;               // free events
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_predict, ev_fill;
    sbo::DevBuf counters;                          // [0]: predictive tiles multiplied

    bool fail(const std::string &m) { err = m; return false; }
};

namespace sbo {

// ---------------------------------------------------------- kernel launchers
// All launchers enqueue on `s` and return hipGetLastError().
// K[i + j*ld] = sf2 exp(-|a_i - b_j|^2 / 2l^2) (+ sn2 on i == j when diag).
hipError_t launch_rbf_fill(hipStream_t s, const float *xa, const float *ya, int64_t ma, const float *xb,
                           const float *yb, int64_t mb, int64_t ld, float ell, float sf2, float sn2, bool diag,
                           float *K);
hipError_t launch_sub_scalar(hipStream_t s, const float *in, float v, int64_t n, float *out);
hipError_t launch_copy_lower(hipStream_t s, const float *src, int64_t ld_src, int64_t n,
                             float *dst, int64_t ld_dst);
// Pack A = sf2 * L^-1 (from an f32 or f64 inverse, lower, column-major) into
// [BK][BM] tiles for row blocks I >= I0 (earlier row blocks are left as they
// are), plus per-k coordinates and sf2 * alpha for all k.
// the two halves of launch_pack_operand (f64 inverse): the operand tiles, and the
// per-k-tile coordinates + sf2 alpha (which waits for alpha)
hipError_t launch_pack_tiles(hipStream_t s, const double *Linv, int64_t ld, int64_t n, int64_t npad, int64_t I0,
                             double sf2, float *aug);
hipError_t launch_pack_kcoord(hipStream_t s, const float *x, const float *y, const float *alpha, int64_t n,
                              int64_t npad, double sf2, float *kcoord);
hipError_t launch_pack_operand(hipStream_t s, const float *Linv, int64_t ld, int64_t n, int64_t npad, int64_t I0,
                               double sf2, const float *x, const float *y, const float *alpha, float *aug,
                               float *kcoord);
hipError_t launch_pack_operand(hipStream_t s, const double *Linv, int64_t ld, int64_t n, int64_t npad, int64_t I0,
                               double sf2, const float *x, const float *y, const float *alpha, float *aug,
                               float *kcoord);
// dst (m x n, f64, ld_dst) = src (f32, ld_src); lower: zero above the diagonal.
hipError_t launch_widen(hipStream_t s, const float *src, int64_t ld_src, int64_t m, int64_t n, bool lower,
                        double *dst, int64_t ld_dst);
// Predictive sweep: part[I][q] = sum over rows of block I of (sf2 L^-1 k_q)^2,
// mean[q] = m0 + sf2 alpha^T k_q.
// Tile cutoff (SkipPlan).  With a tile-norm table (automatic cutoff, one row
// block per workgroup) a workgroup (row block I, query block) bounds tile t's
// share of |dV_I(q)|_2 by 2^(lgn[t]) * K*max(box distance) and drops tiles
// smallest bound first while the dropped bounds sum to at most 2^lg_tau_v
// (binned, fixed point: order-independent); otherwise it drops tile t when
// every K* entry is below 2^-L.  The last row block (which also accumulates
// the mean) keeps every tile within 2^-L_mean.  L >= 150 drops only exact
// zeros (bitwise identical to the dense sweep); L = 0: dense.
// tiles_done (may be null): [0] += number of (BM x BN x BK) tiles multiplied,
// [1] += MFMA products issued on them (prod_full per full tile, 3 / 1 per
// tile at the reduced levels).
struct SkipPlan {
    int L = 0;                  // 0: dense
    int L_mean = 0;             // last row block; <= L means "same as L"
    const float4 *lgn = nullptr;   // per packed tile log2 gain bounds (null: distance test only)
    const float *kcoord = nullptr; // per k-tile coordinates (the |k|_2 bound of the tile-norm test)
    float lg_tau_v = 0.0f;
    int levels = 0;     // with lgn: tiles may run at the reduced precision levels (split sweep)
    int prod_full = 1;  // MFMA products per full-precision tile (6: split sweep), for the counter
    bool records = false;  // also write the split sweep's step records (plan_views' rec)
    bool wide = false;     // empty items' outputs as f64 (the precise sweep's partials and mean)
    int order_blk = 0;     // item order: 0 row-block-major, else blocks of (bi << 8 | bq) -- plan_item
    // rank of a tile's two level increments against drops: log2(time a drop
    // saves / time the level step saves), per-tile sweep time at C4 of six,
    // three, one product(s) 18.6, 12.9, 9.9 ns (variants 22, 20, 21)
    float lvl_key[2] = {0.80f, 1.72f};
};
// The tick's plan (which k-tiles each (row block, query block) item runs,
// non-empty items in row-block-major order, one balanced item range per
// sweep workgroup) in `work` (predict_work_bytes); empty items' outputs are
// written here.  P = sweep workgroups (one per CU).
size_t predict_work_bytes(int64_t npad, int64_t m, int P);
hipError_t launch_plan(hipStream_t s, const float4 *kbox, int64_t npad, const float *qx, const float *qy, int64_t m,
                       int64_t ldp, float ell, float m0, const SkipPlan &skip, float *part, float *mean,
                       unsigned long long *tiles_done, int P, void *work, size_t work_bytes);
// The sweep over the plan in `work` (persistent, P workgroups).
hipError_t launch_predict(hipStream_t s, const float *aug, const float *kcoord, int64_t npad, const float *qx,
                          const float *qy, int64_t m, int64_t ldp, float ell, float m0, float *part, float *mean,
                          int variant, int P, const void *work);
// exp2 coefficient of the RBF kernel: k = exp2(cexp d^2), cexp = -1/(2 l^2 ln 2)
float exp2_coef_f(float ell);
// Per-query sweep work of the plan in `work` (kept k-tiles of the query's
// block summed over row blocks / block size), in the caller's order.
// bcost: (m + kBN - 1) / kBN floats of scratch.
hipError_t launch_plan_cost(hipStream_t s, int64_t npad, int64_t m, int P, const void *work, const int32_t *perm,
                            float *bcost, float *cost);
// The plan's descriptors, tile lists and per-workgroup ranges inside `work`.
void plan_views(int64_t npad, int64_t m, int P, const void *work, const int4 **desc, const unsigned short **tl,
                const int **seg, const int4 **rec = nullptr);
// Split-operand (bf16 x3) predictive sweep, predict_x3.hip: the packed
// operand split into three bf16 planes per half-tile and the per-k-tile
// coordinates in natural order, for row blocks >= I0 (coordinates: all).
size_t x3_operand_bytes(int64_t npad);
size_t x3_coord_bytes(int64_t npad);
// (ax3 null: the coordinates only; kc3 null: the planes only)
hipError_t launch_pack_x3(hipStream_t s, const float *aug, const float *kcoord, int64_t npad, int64_t I0, int wide,
                          char *ax3, float *kc3);
// the split operand's layout a kernel variant reads (1: the wide 32x32x16 shape)
// tile-list entry of the plan: k-tile index | precision level code << kLevelShift
constexpr int kLevelShift = 14;
// Step record of the split sweep (plan_rec_kernel), one int4 per kept tile in
// sweep order: x = the packed tile's offset in the split operand (KiB, two
// half-tiles of 48), y = its k-tile's coordinate offset in kc3 (floats),
// z = query block, w = row block | level code << 16 | first / last tile of
// its item (kRecFirst, kRecLast).
constexpr int kRecFirst = 1 << 20, kRecLast = 1 << 21;
// the split sweeps that honour the plan's precision levels
inline bool x3_levels(int variant) { return variant == 3 || variant == 23 || variant == 24 || variant == 30 || variant == 32 || variant == 33 || variant == 39 || variant == 41 || variant == 42 || variant == 43 || variant == 46 || variant == 47 || variant == 48 || variant == 49 || variant == 51 || variant == 52 || variant == 53 || variant == 54 || variant == 55 || variant == 56 || variant == 57 || (variant >= 58 && variant <= 61); }
// Sweeps the product library accepts (all compute the full result; 3 is the
// default).  The timing diagnostics (parts of the work left out, forced
// precision levels, phase stamps) exist only in the diagnostic build
// (-DSBO_DIAG, lib/libsbo_diag.so, selected by SBO_LIB for tools/).
inline bool variant_allowed(int v) {
#ifdef SBO_DIAG
    return v >= 0 && v <= 61;
#else
    return v == 0 || v == 1 || v == 3 || v == 22;
#endif
}
inline int x3_layout(int variant) { return (variant == 13 || variant == 14) ? 1 : 0; }
// The sweep over the plan with the split operand; qx/qy must be readable in
// whole 128-query blocks (padded to round_up(m, kBN)).  variant: 2 (4-7:
// timing diagnostics with parts of the work left out).
// Diagnostic build (SBO_OPT_KERNEL_VARIANT 39): summed phase cycles of the
// split sweep since the last read (see g_x3_stamps), then reset.
hipError_t read_x3_stamps(double *out, int n);
hipError_t launch_predict_x3(hipStream_t s, const char *ax3, const float *kc3, const int4 *desc, const int4 *rec,
                             const int *seg, int P, int n_items, int nI, const float *qx, const float *qy, int64_t m,
                             int64_t ldp, float cexp, float m0, float *part, float *mean, int variant);
// lgn[2 (tile_start(I) + t)] = log2 bounds (16 max row 1-norm, spectral,
// Frobenius) of A_It, lgn[2 (..) + 1] = (16 max row 1-norm, spectral) of its
// bf16 pieces A1 and A2 (f64 sums, rounded up) for row blocks I >= I0 (-1000
// for an all-zero matrix).
hipError_t launch_tile_norms(hipStream_t s, const float *aug, int64_t npad, int64_t I0, float4 *lgn);
// the f64 operand's pack (launch_pack_tiles) and the tile norms in one pass
hipError_t launch_pack_tile_norms(hipStream_t s, const double *Linv, int64_t ld, int64_t n, int64_t npad, int64_t I0,
                                  double sf2, float *aug, float4 *lgn);
// Blocked Cholesky: factor the kb x kb diagonal block at A (column-major,
// lda = ld) of step k0 in place (kb <= kCholNB); info as rocSOLVER's.
constexpr int kCholNB = 128;
// version 1: chol_diag_mfma_kernel (16-column panels, MFMA trailing updates; default), 0: chol_diag_kernel
hipError_t launch_chol_diag(hipStream_t s, float *A, int64_t ld, int kb, int64_t k0, int *info, int version = 1);
// C -= P Q^T over 128 x 128 tiles (lower: the tiles on and below the diagonal of an m x m C), f32, lda ld, K columns
hipError_t launch_chol_update(hipStream_t s, const float *P, const float *Q, int64_t ld, int64_t m, int64_t nc,
                              int64_t K, bool lower, float *C);
// SBO_OPT_CHOL_GEMM 3 (csrc/chol_x3.hip): the outer panel P (m x K f32, lda ld,
// K a multiple of 32) into three bf16 planes in MFMA fragment order
// (chol_x3_bytes), then C (rows x cols, lda ld) -= P[r0 ..] P[c0 ..]^T on the bf16
// matrix cores with six split products per f32 product (lower: the tiles on and
// below the diagonal of a square region with r0 == c0)
size_t chol_x3_bytes(int64_t m, int64_t K);
hipError_t launch_chol_split(hipStream_t s, const float *P, int64_t ld, int64_t m, int64_t K, char *planes);
hipError_t launch_chol_update_x3(hipStream_t s, const char *planes, int64_t m, int64_t K, int64_t r0, int64_t rows,
                                 int64_t c0, int64_t cols, bool lower, float *C, int64_t ld);
// The panel below it: A21 (m2 x kb, lda ld) := A21 L11^-T (forward substitution, f32).
// version 1: chol_trsm_mfma_kernel (MFMA updates of the later columns; default), 0: chol_trsm_kernel (bitwise equal)
hipError_t launch_chol_trsm(hipStream_t s, const float *L11, int64_t ld, int kb, float *A21, int64_t m2, int version = 1);
// d = (double)in - v;  out = (float)d
hipError_t launch_widen_sub(hipStream_t s, const float *in, double v, int64_t n, double *d);
// alpha = X^T X (obs - m0) from the f64 inverse X (lower, lda ld), z = X (obs -
// m0) kept; work: alpha_work_bytes(n) (the first pass's per-chunk partials)
size_t alpha_work_bytes(int64_t n);
hipError_t launch_alpha_f64(hipStream_t s, const double *X, int64_t ld, int64_t n, const float *obs, double m0,
                            double *z, double *alpha, double *work);
hipError_t launch_narrow(hipStream_t s, const double *d, int64_t n, float *out);
// out[r] = sum_c A[r + c ld] x[c] (c < n) for rows r < rows of a column-major f64 matrix
hipError_t launch_row_dot(hipStream_t s, const double *A, int64_t ld, int64_t rows, int64_t n, const double *x,
                          double *out);
// out[i + j ldo] = (float)d[i + j ldd], i < m, j < n
hipError_t launch_narrow_2d(hipStream_t s, const double *d, int64_t ldd, int64_t m, int64_t n, float *out,
                            int64_t ldo);
// out[j * stride] = (float)d[j], j < n
hipError_t launch_narrow_strided(hipStream_t s, const double *d, int64_t n, float *out, int64_t stride);
// row_l1[i] = sum_j |A_ij| over the packed operand (f64), rows of row blocks >= I0.
hipError_t launch_row_l1(hipStream_t s, const float *aug, int64_t npad, int64_t I0, double *row_l1);
// Per k-tile bounding boxes of the (internally ordered) training points.
hipError_t launch_tile_boxes(hipStream_t s, const float *x, const float *y, int64_t n, int64_t npad,
                             float4 *kbox);
// Acquisition over predictive partials (fused reduce + sets + block argmax).
// perm (may be null): sweep position i holds caller query perm[i]; outputs and
// key indices are written in the caller's order.
hipError_t launch_acquire(hipStream_t s, const float *part, const float *mean, int nI, int64_t ldp,
                          int64_t m, float sf2, double beta, double f_min, int score_kind,
                          int64_t index_offset, const int32_t *perm, float *mu, float *sd, double *lo,
                          double *hi, uint8_t *safe, sbo_key *block_keys);
// the same over the precise sweep's f64 partials and mean (sf2 in f64)
hipError_t launch_acquire(hipStream_t s, const double *part, const double *mean, int nI, int64_t ldp,
                          int64_t m, double sf2, double beta, double f_min, int score_kind,
                          int64_t index_offset, const int32_t *perm, float *mu, float *sd, double *lo,
                          double *hi, uint8_t *safe, sbo_key *block_keys);
// Precise sweep (predict_f64.hip, SBO_OPT_PRECISION): A = sf2 L^-1 packed in
// f64 from the fit's f64 inverse for row blocks >= I0 (tile (I, t) at
// tile_start(I) + t, two 64 KiB stages in MFMA fragment order), and per k-tile
// half the f64 x, y, sf2 alpha (alpha from the f64 solve).
size_t f64_operand_bytes(int64_t npad);
size_t f64_coord_bytes(int64_t npad);
hipError_t launch_pack_f64(hipStream_t s, const double *Linv, int64_t ld, int64_t n, int64_t npad, int64_t I0,
                           double sf2, const float *x, const float *y, const double *alpha, double *a64,
                           double *kc64);
// The sweep over the plan (descriptors and tile lists of plan_views; every
// kept tile in f64): part[I][q] (f64) = sum over row block I of V^2, mean[q]
// (f64) = m0 + sf2 alpha^T k_q.
hipError_t launch_predict_f64(hipStream_t s, const double *a64, const double *kc64, const int4 *desc,
                              const unsigned short *tl, const int *seg, int P, int n_items, int nI, const float *qx,
                              const float *qy, int64_t m, int64_t ldp, double ell, double m0, double *part,
                              double *mean);
// The int8 sliced precise sweep (predict_oz.hip, SBO_OPT_PRECISE_KERNEL 1):
// A = sf2 L^-1 from the fit's f64 inverse as five balanced base-256 int8
// digit slices per 16-row block and k-tile (80 KiB per packed tile) with a
// power-of-two exponent per block (oz_exp_bytes: 16 int32 per tile), per
// k-tile x, y (f64 and f32) and sf2 alpha (f64).  The sweep reads the same plan as launch_predict_f64 and
// writes the same f64 partials and mean.
size_t oz_operand_bytes(int64_t npad);
size_t oz_exp_bytes(int64_t npad);
size_t oz_coord_bytes(int64_t npad);
hipError_t launch_pack_oz(hipStream_t s, const double *Linv, int64_t ld, int64_t n, int64_t npad, int64_t I0,
                          double sf2, const float *x, const float *y, const double *alpha, char *aoz, int *eoz,
                          char *koz, bool pairs = false);
hipError_t launch_predict_oz(hipStream_t s, const char *aoz, const int *eoz, const char *koz, const int4 *desc,
                             const unsigned short *tl, const int *seg, int P, int n_items, int nI, const float *qx,
                             const float *qy, int64_t m, int64_t ldp, double ell, double m0, double *part,
                             double *mean, int variant = 1, const char *kzt = nullptr);
// The K* table (SBO_OPT_PRECISE_KERNEL 3): bytes per query block, and the
// table of nq query blocks of the queries qx/qy (m of them) for every k-tile.
// pairs (SBO_OPT_PRECISE_KERNEL 4): exponents shared by k-tile pairs (2p,
// 2p + 1) -- the operand (launch_pack_oz), the table and the sweep (variant 4)
size_t oz_table_bytes(int64_t npad, bool pairs = false);
hipError_t launch_kstar_table(hipStream_t s, const char *koz, const float *qx, const float *qy, int64_t m,
                              int64_t npad, double ell, int64_t nq, char *kzt, bool pairs = false);
// The int8-sliced f64 GEMM (ozgemm.hip): C (m x n, ldc) = alpha op(A) op(B)
// (+ C), column-major f64, op(A) m x K (A itself K x m with kGzTransA), op(B)
// K x n (n x K with kGzTransB); a triangular operand's zero part is not read;
// kGzTransC stores C^T (C then points at n x m storage, ldc its leading
// dimension); nd digits (5, 6); K <= 16384; workspace of
// gz_workspace_bytes(m, n, K, nd).
constexpr unsigned kGzTriA = 1;        // op(A) lower triangular: a_ik = 0 for k > i
constexpr unsigned kGzTransA = 2;
constexpr unsigned kGzTriBLower = 4;   // op(B) lower triangular: b_kj = 0 for k < j
constexpr unsigned kGzTriBUpper = 8;   // op(B) upper triangular: b_kj = 0 for k > j
constexpr unsigned kGzTransB = 16;
constexpr unsigned kGzTransC = 32;
constexpr unsigned kGzBeta1 = 64;      // C += instead of C =
constexpr unsigned kGzLowerC = 128;    // (f32 form) only tiles that meet C's lower triangle
size_t gz_workspace_bytes(int64_t m, int64_t n, int64_t K, int nd);
hipError_t launch_gz_gemm(hipStream_t s, int nd, const double *A, int64_t lda, const double *B, int64_t ldb,
                          int64_t m, int64_t n, int64_t K, double alpha, double *C, int64_t ldc, unsigned flags,
                          char *ws);
// The same product on f32 operands and an f32 C (4 or 5 digits: the Cholesky's
// updates, SBO_OPT_CHOL_GEMM 4 / 5); kGzLowerC skips the tiles above C's diagonal.
hipError_t launch_gz_gemm_f32(hipStream_t s, int nd, const float *A, int64_t lda, const float *B, int64_t ldb,
                              int64_t m, int64_t n, int64_t K, double alpha, float *C, int64_t ldc, unsigned flags,
                              char *ws);
// ... and with one pack of the panel's m rows shared by every product of an
// outer step: op(A) its rows a0 .., op(B)^T its rows b0 .. (multiples of 128)
size_t gz_pack_bytes(int64_t m, int64_t K, int nd);
hipError_t launch_gz_pack_f32(hipStream_t s, int nd, const float *P, int64_t ld, int64_t m, int64_t K, char *pack);
hipError_t launch_gz_gemm_packed_f32(hipStream_t s, int nd, const char *pack, int64_t mpack, int64_t K, int64_t a0,
                                     int64_t m, int64_t b0, int64_t n, double alpha, float *C, int64_t ldc,
                                     unsigned flags);
// The fit's accuracy guard of the f64 inverse (inv_check.hip): on kChkQ - 1
// queries (coordinates at *qxy: x[kChkQ] then y[kChkQ], filled by the caller
// before the launch) plus the residual r = obs - m0 as the last right-hand
// side, V0 = Linv Kq and one refinement against the f32 factor L, dV = Linv
// (Kq - L V0), both lower-triangular column-major with lda ld; *colsums = per
// query column (sum dV (2 V0 + dV), sum (V0 + dV)^2, sum V0 z0, sum V0 dz +
// dV z0 + dV dz) with z0 / dz the residual's columns.  work:
// inv_check_bytes(n); with Linv null only the pointers are set.
constexpr int kChkQ = 32;
int64_t inv_check_rows(int64_t n);
size_t inv_check_bytes(int64_t n);
hipError_t launch_inv_check(hipStream_t s, const double *Linv, const float *L, int64_t ld, int64_t n,
                            const float *x, const float *y, const float *obs, double m0, double sf2, double ell,
                            void *work, float **qxy, double **colsums);
// Morton ordering of the queries (query_order.hip): workspace of
// query_order_bytes(m); returns the permutation and the gathered coordinates
// (all inside the workspace).
size_t query_order_bytes(int64_t m);
hipError_t launch_query_order(hipStream_t s, const float *qx, const float *qy, int64_t m, const float bbox[4],
                              void *work, size_t work_bytes, int32_t **perm, float **sqx, float **sqy);
// Raster-grid queries (query_order.hip): blocks of kGridPatchFast points
// along the grid's fast axis x kGridPatchSlow rows, patches in raster order,
// padded positions with perm = -1.  launch_grid_detect (workspace
// query_grid_bytes(m), synchronizes the stream) reads the raster's shape;
// grid_layout turns it into a layout (false: not a raster, or more padding
// than grid_max_positions allows -- Morton then); launch_query_grid
// gathers the q.ms sweep positions.
size_t query_grid_bytes(int64_t m);
hipError_t launch_grid_detect(hipStream_t s, const float *qx, const float *qy, int64_t m, void *work,
                              unsigned long long host_g[6]);
bool grid_layout(const unsigned long long g[6], int64_t m, QueryGrid &q);
hipError_t launch_query_grid(hipStream_t s, const float *qx, const float *qy, int64_t m, const QueryGrid &q,
                             void *work, int32_t **perm, float **sqx, float **sqy);
// ComputeSets from given mu/sd (staged API).
hipError_t launch_sets(hipStream_t s, const float *mu, const float *sd, int64_t m, double beta,
                       double f_min, double *lo, double *hi, uint8_t *safe);
hipError_t launch_sets(hipStream_t s, const double *mu, const double *sd, int64_t m, double beta,
                       double f_min, double *lo, double *hi, uint8_t *safe);
// Masked argmax over f64 scores -> block keys.
hipError_t launch_argmax_blocks(hipStream_t s, const double *score, const uint8_t *mask, int64_t m,
                                int64_t index_offset, sbo_key *block_keys);
// Reduce nblocks keys into *out (device pointer).
hipError_t launch_reduce_keys(hipStream_t s, const sbo_key *keys, int64_t nblocks, sbo_key *out);

inline int64_t acq_blocks(int64_t m) { return (m + kAcqThreads - 1) / kAcqThreads; }

// ------------------------------------------------------ frontier (8(f)1)
// Device raster of FindSafetyContourIndices (:425-475): the node's
// int-truncated bounds from a device min/max, each grid point's pixel
// (scaled by width/height, out-of-range dropped), last writer (highest
// index) wins -- atomicMax on a dense owner map, which replaces the node's
// unordered_map (:468-475) -- and owner[k] = that point if it is safe, else
// -1 (a pixel is foreground exactly when its last writer is safe).
// img[k] = 1 on foreground pixels.  Workspace: frontier_work_bytes(m);
// owner: width*height int32; img: width*height bytes.
size_t frontier_work_bytes(int64_t m);
hipError_t launch_frontier_raster(hipStream_t s, const double *Dx, const double *Dy, const uint8_t *safe, int64_t m,
                                  int width, int height, void *work, int32_t *owner, uint8_t *img);
// F[i] = owner[pix[i]]; when lo is non-null also out[c*nf + i] = (Dx, Dy, lo, hi)[F[i]].
hipError_t launch_frontier_gather(hipStream_t s, const int32_t *pix, int64_t nf, const int32_t *owner,
                                  const double *Dx, const double *Dy, const double *lo, const double *hi, int32_t *F,
                                  double *out);
// host side (frontier.cpp)
void trace_external_pixels(const uint8_t *img, int w, int h, std::vector<int32_t> &pix);
int64_t select_subgoal(size_t nf, const double *fx, const double *fy, const double *flo, const double *fhi,
                       double goal_x, double goal_y);

}  // namespace sbo
