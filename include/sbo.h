/*
 * sbo.h -- C ABI of the MI355X safe-BO planning-tick library (libsbo.so).
 *
 * The reference has no plugin/FFI API for this path.  Its
 * boundary is (i) the GetTerrainMapWithUncertainty service between the
 * external GP mapper and the node, consumed at
 * src/safe_bayesian_optimization_node.cpp:576-647 (request resolution[2] f32
 * :580-581; response success, message, n_width_cells, n_height_cells,
 * x_coords[], y_coords[], values[] (= mu), uncertainties[] (= sigma)
 * :606-644), and (ii) the node's private calls ComputeSets() (:399-416),
 * FindSafetyContourIndices() (:418-497) and GetNextSubgoal() (:499-550).
 * Each entry point below names the reference interface it replaces.
 *
 * Conventions (mirroring the reference, :129-177, :503-506, :1503):
 *   - the caller owns every buffer; no exceptions cross this boundary;
 *   - one context per thread; a context is not thread-safe;
 *   - calls are synchronous with respect to the context's HIP stream unless
 *     SBO_ASYNC is passed (then results are ready when the stream drains);
 *   - array pointers are host pointers unless SBO_DEVICE_PTRS is passed, in
 *     which case EVERY array argument of that call is a device pointer;
 *   - coordinates are SoA (all x, then all y), like the column-major
 *     Eigen::Matrix<double,Dynamic,2> D_ (:132);
 *   - "no subgoal" is -1 (:503-506).
 */
#ifndef SBO_H_
#define SBO_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SBO_API __attribute__((visibility("default")))

typedef enum sbo_status {
    SBO_OK = 0,
    SBO_E_INVAL = 1,    /* bad argument (null pointer, n <= 0, bad hyper-parameter) */
    SBO_E_NOT_SPD = 2,  /* the Cholesky's leading minor (rocSOLVER info convention): K not positive definite */
    SBO_E_DEVICE = 3,   /* HIP / rocBLAS / rocSOLVER runtime error */
    SBO_E_OOM = 4,      /* device allocation failed */
    SBO_E_EMPTY = 5,    /* nothing to operate on (no fit yet, empty input) */
    SBO_E_STATE = 6     /* call out of order (e.g. predict before fit) */
} sbo_status;

/* flags */
#define SBO_DEVICE_PTRS 0x1u  /* all array arguments are device pointers */
#define SBO_ASYNC 0x2u        /* do not synchronise the stream before returning */

/* GP hyper-parameters (config/lpsc.yaml:35-37: noise_level 0.1,
 * length_scale 0.4, sigma_f 1.0).  noise_level is a noise VARIANCE. */
typedef struct sbo_hyper {
    double length_scale;
    double sigma_f;
    double noise_level;
    double prior_mean;
} sbo_hyper;

/* Acquisition score for the grid argmax (a10). */
typedef enum sbo_score {
    SBO_SCORE_WIDTH = 0,  /* Q(:,1) - Q(:,0), the width GetNextSubgoal ranks (:516) */
    SBO_SCORE_UCB = 1     /* Q(:,1) = mu + beta*sigma */
} sbo_score;

/* Result of a masked argmax: highest score, lowest global index on ties.
 * idx = -1 when no point is eligible.  Keys from different shards combine
 * with sbo_key_combine (this is what crosses ranks). */
typedef struct sbo_key {
    double score;
    int64_t idx;
} sbo_key;

typedef struct sbo_ctx sbo_ctx;

/* Library / context ------------------------------------------------------ */
SBO_API const char *sbo_version(void);
SBO_API const char *sbo_status_string(sbo_status s);
/* Replaces the node's service client (:75-77): binds a HIP device.  */
SBO_API sbo_status sbo_create(int device, sbo_ctx **out);
SBO_API void sbo_destroy(sbo_ctx *ctx);
/* Run on the caller's HIP stream (hipStream_t), e.g. torch's current stream.
 * NULL restores the context's own stream. */
SBO_API sbo_status sbo_set_stream(sbo_ctx *ctx, void *hip_stream);
SBO_API const char *sbo_last_error(const sbo_ctx *ctx);

/* GP mapper (the external terrain_mapping_node, a1+a2) -------------------
 * Fit the posterior to n measurements (x, y, obs): RBF fill (HIP kernel),
 * the library's blocked Cholesky (SBO_OPT_CHOLESKY), L^-1 in f64 by its block
 * recursion (SBO_OPT_INVERSE), alpha = L^-T L^-1 (y - m0) from that inverse,
 * the packed predictive operand and its tile bounds, and the precision probe
 * (SBO_OPT_PRECISION).  Replaces the mapper's fit behind the service. */
SBO_API sbo_status sbo_fit(sbo_ctx *ctx, const float *x, const float *y, const float *obs,
                           int64_t n, sbo_hyper hyper, uint32_t flags);

/* Streaming update (C5): append b measurements with a block Cholesky update
 * (L21 = K21 L11^-T, L22 = chol(K22 - L21 L21^T)), then re-solve alpha.
 * Replaces a full re-fit on each spatial_data_size change (:552-566). */
SBO_API sbo_status sbo_append(sbo_ctx *ctx, const float *x, const float *y, const float *obs,
                              int64_t b, uint32_t flags);

/* Number of training points currently fitted (0 before sbo_fit). */
SBO_API int64_t sbo_num_train(const sbo_ctx *ctx);

/* Predict (a3+a4): posterior mean and latent std at m query points
 * (the service's values[] and uncertainties[], :642-643).  mu/sd may be NULL
 * to skip that output. */
SBO_API sbo_status sbo_predict(sbo_ctx *ctx, const float *qx, const float *qy, int64_t m,
                               float *mu, float *sd, uint32_t flags);

/* ComputeSets() (:399-416) == ComputeConfidenceIntervals + UpdateSafeSet:
 *   c = beta*sd;  lo = mu - c;  hi = mu + c;  safe = lo > f_min
 * evaluated in IEEE double exactly as the node's Eigen code (no FMA).
 * lo/hi are Q_.col(0)/Q_.col(1) (f64), safe is S_ (1 byte per point). */
SBO_API sbo_status sbo_compute_sets(sbo_ctx *ctx, const float *mu, const float *sd, int64_t m,
                                    double beta, double f_min, double *lo, double *hi,
                                    uint8_t *safe, uint32_t flags);
/* The same on f64 inputs: the node's own mu_/std_ (Eigen::VectorXd,
 * node.cpp:129-130, filled at :641-643) passed as they are -- lossless for
 * any service value, bit-exact with ComputeSets() (:411-416). */
SBO_API sbo_status sbo_compute_sets_f64(sbo_ctx *ctx, const double *mu, const double *sd, int64_t m,
                                        double beta, double f_min, double *lo, double *hi,
                                        uint8_t *safe, uint32_t flags);

/* Grid acquisition argmax (a10): argmax of score over mask (mask may be NULL),
 * lowest index on ties, NaN never wins.  index_offset is added to local
 * indices (the first global row of this rank's shard). */
SBO_API sbo_status sbo_argmax(sbo_ctx *ctx, const double *score, const uint8_t *mask, int64_t m,
                              int64_t index_offset, sbo_key *out, uint32_t flags);

/* The whole planning tick on one shard of the grid, fused on the device:
 * predict -> ComputeSets -> masked argmax of `score` over the safe set.
 * Output arrays may be NULL to skip writing them (the key is always produced).
 * This is the headline step measured by bench.py. */
SBO_API sbo_status sbo_tick(sbo_ctx *ctx, const float *qx, const float *qy, int64_t m,
                            double beta, double f_min, sbo_score score, int64_t index_offset,
                            float *mu, float *sd, double *lo, double *hi, uint8_t *safe,
                            sbo_key *out, uint32_t flags);

/* Sweep work of each query under the current fit: builds the tick's tile
 * plan for these queries (no sweep) and writes cost[i] = the k-tiles its
 * 128-query block multiplies, summed over row blocks and weighted by their
 * precision level's sweep time (1, 42/64, 33/64 for six, three, one
 * product(s)), / the block's size, in the caller's order.  For cost-balanced M-sharding across ranks (every
 * rank computes the same costs from the same inputs: the plan is
 * deterministic); no reference counterpart. */
SBO_API sbo_status sbo_query_cost(sbo_ctx *ctx, const float *qx, const float *qy, int64_t m, float *cost,
                                  uint32_t flags);

/* Combine two shard keys (the cross-rank reduction of sbo_tick / sbo_argmax). */
SBO_API sbo_key sbo_key_combine(sbo_key a, sbo_key b);

/* Reduce n keys (e.g. the P keys of a cross-rank all-gather) to one by the
 * sbo_key_combine rule.  With SBO_DEVICE_PTRS keys and out are device
 * pointers and the reduction is one workgroup on the context's stream (with
 * SBO_ASYNC nothing synchronises: the combined key stays on the device, so a
 * sharded tick needs no host round trip per step); otherwise host memory. */
SBO_API sbo_status sbo_keys_reduce(sbo_ctx *ctx, const sbo_key *keys, int64_t n, sbo_key *out, uint32_t flags);

/* Host-side node logic (no device needed) ---------------------------------
 * FindSafetyContourIndices() (:418-497): rasterise safe into a
 * height x width image with the node's int-truncated bounds, trace external
 * contours (cv::findContours RETR_EXTERNAL, CHAIN_APPROX_NONE restated) and
 * map contour pixels back to grid indices (last writer wins, duplicates kept).
 * Dx/Dy are D_.col(0)/D_.col(1) (f64).  Writes at most out_cap indices,
 * stores the total in *count; returns SBO_E_INVAL if out_cap was too small. */
SBO_API sbo_status sbo_find_safety_contour_indices(const double *Dx, const double *Dy,
                                                   const uint8_t *safe, int64_t m,
                                                   int width_cells, int height_cells,
                                                   int32_t *out, int64_t out_cap, int64_t *count);

/* GetNextSubgoal() (:499-550): frontier, distance sort to the goal, top
 * max(1, F/4), strict-> argmax of Q(:,1)-Q(:,0).  Returns the grid index or -1. */
SBO_API int64_t sbo_next_subgoal(const double *Dx, const double *Dy, const double *lo,
                                 const double *hi, const uint8_t *safe, int64_t m,
                                 int width_cells, int height_cells, double goal_x, double goal_y);

/* The same two steps on device-resident grid data: with
 * SBO_DEVICE_PTRS, Dx/Dy/lo/hi/safe are device arrays (e.g. the tick's own
 * outputs); the O(M) raster -- bounds, pixel arithmetic, the last-writer
 * maps -- runs on the GPU and only the width x height image crosses to the
 * host for the border follow.  Results are identical to the host functions
 * above for finite coordinates (non-finite ones: the device bounds ignore
 * them).  Without the flag they call the host functions.  `out` is host
 * memory; count receives the frontier size even when out_cap is too small
 * (SBO_E_INVAL).  *index = -1 when there is no frontier. */
SBO_API sbo_status sbo_frontier(sbo_ctx *ctx, const double *Dx, const double *Dy, const uint8_t *safe,
                                int64_t m, int width_cells, int height_cells, int32_t *out,
                                int64_t out_cap, int64_t *count, uint32_t flags);
SBO_API sbo_status sbo_subgoal(sbo_ctx *ctx, const double *Dx, const double *Dy, const double *lo,
                               const double *hi, const uint8_t *safe, int64_t m, int width_cells,
                               int height_cells, double goal_x, double goal_y, int64_t *index,
                               uint32_t flags);

/* Post-selection geometry, host, f64.  Rings are the
 * exterior ring as Boost stores it: x[] / y[], closing point included.
 * sbo_polygon_correct: bg::correct for polygon<point, false, true> (the
 * node's :682): closes an open ring (needs cap >= n + 1) and reverses a
 * clockwise one; *n_out = new length.
 * sbo_polydist: polydist (src/libraries/polygeom_lib.cpp:401-474) including
 * its nearest-vertex quirk (:439-440); SBO_E_EMPTY for fewer than 2 ring
 * points, with the reference's intended dist 1e8 and point (0, 0).
 * sbo_point_within: bg::within(point, polygon) (:657), 1 strictly inside,
 * 0 outside or on the boundary.
 * sbo_project_subgoal: the node's step after GetNextSubgoal (:651-704): the
 * goal when within the ring (returns 1); else (Dx, Dy)[subgoal_index]
 * projected by polydist onto the corrected ring (returns 0); -1 when there
 * is no subgoal (index < 0) or the ring is empty. */
SBO_API sbo_status sbo_polygon_correct(double *rx, double *ry, int64_t n, int64_t cap, int64_t *n_out);
SBO_API sbo_status sbo_polydist(const double *rx, const double *ry, int64_t n, double px, double py,
                                double *proj_x, double *proj_y, double *dist);
SBO_API int sbo_point_within(const double *rx, const double *ry, int64_t n, double px, double py);
SBO_API int sbo_project_subgoal(const double *rx, const double *ry, int64_t n, double goal_x, double goal_y,
                                int64_t subgoal_index, const double *Dx, const double *Dy, int64_t m,
                                double *out_x, double *out_y, double *out_dist);

/* Bounding box of the fitted training points (x0, x1, y0, y1), widened by
 * every sbo_append and carried through sbo_export_state / sbo_import_state:
 * the extent the service grid spans by default (mapper side of :583-586).
 * SBO_E_STATE before the first fit. */
SBO_API sbo_status sbo_get_bounds(const sbo_ctx *ctx, double *bounds);

/* The diagonal jitter added by SBO_OPT_JITTER_RETRIES to the current fit
 * (0.0 when the first factorization succeeded).  SBO_E_STATE before a fit. */
SBO_API sbo_status sbo_get_jitter(const sbo_ctx *ctx, double *jitter);

/* Fitted predictive state as one device blob (fit on one
 * rank, broadcast the operand to the others instead of refitting there).
 * sbo_state_bytes gives the size (the packed sf2 L^-1 tiles dominate:
 * ~2 N^2 B), sbo_export_state writes it into a caller device buffer,
 * sbo_import_state restores it into another context on any device.  An
 * imported context predicts, ticks and reports like the original (bitwise
 * identical sweeps) but holds no factor: sbo_append / sbo_get_factor return
 * SBO_E_STATE until the next sbo_fit.  sbo_import_state rejects
 * (SBO_E_INVAL) a blob whose magic, size, section offsets, header fields
 * or training order do not match what (n, npad) implies. */
SBO_API sbo_status sbo_state_bytes(sbo_ctx *ctx, int64_t *bytes);
SBO_API sbo_status sbo_export_state(sbo_ctx *ctx, void *dev_buf, int64_t cap);
SBO_API sbo_status sbo_import_state(sbo_ctx *ctx, const void *dev_buf, int64_t bytes);

/* Raw border follower used by the frontier: img is height x width u8
 * row-major; points (x,y) pairs; start[c]..start[c+1] bound contour c.
 * Returns the number of contours, or -1 if a capacity was exceeded. */
SBO_API int64_t sbo_find_contours_external(const uint8_t *img, int width, int height,
                                           int32_t *pts, int64_t pts_cap,
                                           int64_t *start, int64_t contours_cap);

/* Staged-parity accessors (tests) ----------------------------------------
 * RBF fill alone (a1): writes the n x n column-major K (lda = n). */
SBO_API sbo_status sbo_rbf_fill(sbo_ctx *ctx, const float *x, const float *y, int64_t n,
                                sbo_hyper hyper, float *K, uint32_t flags);
/* Copy out the current factor L (n x n column-major, lower; upper part
 * zeroed) and alpha (n), both in the internal training order (sbo_get_order). */
SBO_API sbo_status sbo_get_factor(sbo_ctx *ctx, float *L, float *alpha, uint32_t flags);

/* The k-d order sbo_fit stores host points in (SBO_OPT_SPATIAL_ORDER 3):
 * perm[j] = the caller's index of stored row j, for n points whose first lands
 * at position first_offset of a 64-point k-tile (0 for a fit; sbo_append's
 * batch starts at the current N).  Host pointers, no context, no device. */
SBO_API sbo_status sbo_kd_order(const float *x, const float *y, int64_t n, int64_t first_offset, int64_t *perm);

/* Options.  SBO_OPT_INVERSE_BITS (32 | 64, default 64): precision in which
 * L^-1 is computed before sf2 * L^-1 is rounded to f32 for the predictive
 * sweep (64 = widen L, rocsolver_dtrtri; 32 = rocsolver_strtri).  Takes
 * effect at the next sbo_fit / sbo_append. */
#define SBO_OPT_INVERSE_BITS 1
/* SBO_OPT_SPATIAL_ORDER (0 caller order | 1 Hilbert | 2 Morton | 3 k-d,
 * default 3): store the training points spatially sorted (sbo_fit sorts all
 * points, sbo_append sorts each batch), so every 64-point k-tile of the
 * predictive sweep is spatially compact -- Hilbert: no Morton jumps inside
 * a tile (12 % fewer tiles pass the cutoff at C3 than Morton); k-d:
 * recursive bisection across the longer side into whole k-tiles, 16 %
 * smaller tile boxes than Hilbert on scattered points (C4 sweep 23.5 ->
 * 22.4 ms).  The
 * posterior does not depend on the order; sbo_get_factor returns the factor
 * of the internally ordered K and sbo_get_order the caller's index of each
 * internal row.  Takes effect at the next sbo_fit / sbo_append. */
#define SBO_OPT_SPATIAL_ORDER 2
/* SBO_OPT_TILE_SKIP (-1 | 0 | L in [16, 1000], default -1): skip a k-tile
 * for a workgroup of queries when the two bounding boxes are so far apart
 * that every K* entry of the block is below 2^-L (|d| > l sqrt(2 L ln 2)).
 * 0: dense sweep.  L >= 150: the dropped entries are exactly +0.0 in f32 and
 * the result is bitwise identical to the dense sweep.  -1 (auto): L is the
 * smallest exponent whose worst-case effect -- 2^-L max_i |(sf2 L^-1)_i|_1 on
 * any V entry, hence 2 sqrt(N sf2) times that on sigma^2, and
 * 2^-L |sf2 alpha|_1 on any mean -- stays below 2^-B sf2 (resp. 2^-B
 * sqrt(sf2)), B = SBO_OPT_SKIP_BUDGET, computed from the fitted factor
 * (sbo_get_skip reports it). */
#define SBO_OPT_TILE_SKIP 3
/* SBO_OPT_QUERY_ORDER (0 | 1 | 2, default 1): the order the queries of a
 * tick are swept in, so that each workgroup's 128 queries are spatially
 * compact and skip more k-tiles -- 0 the caller's order; 2 Morton order
 * (device radix sort, ~0.1 ms per 10^6 points); 1 (default) 8 x 16 grid
 * patches when the queries are a raster grid (rows of one coordinate, the
 * other repeating row by row; a contiguous run of rows cut anywhere
 * qualifies; detected with one stream synchronization per new query
 * buffer, and the patch layout is a valid order for whatever the buffer
 * later holds), else Morton order.  Outputs and argmax indices stay in the
 * caller's order. */
#define SBO_OPT_QUERY_ORDER 4
/* SBO_OPT_KERNEL_VARIANT, the predictive sweep: 3 (default) = split
 * operands on bf16 MFMA -- sf2 L^-1 and K* as three bf16 pieces each, up to
 * six v_mfma_f32_16x16x32_bf16 products per f32 product, f32 accumulation,
 * eight waves per CU; with the automatic cutoff the tile plan runs tiles
 * whose share of the variance is small at three or one product(s), charged
 * to the same error budget as the skipped tiles (SBO_OPT_SKIP_BUDGET);
 * 22 = variant 3 with every kept tile at six products (f32-accurate:
 * variance error vs a host f64 sweep 5.07e-6 at N = 16384 against 5.00e-6
 * for variant 0); 2 = variant 22 with four waves of 32 queries; 0 = f32
 * MFMA (16x16x4) with an f32 cross-tile accumulator; 1 = variant 0 with an
 * f64 one; 9, 10 = variant 22 with the A stage issued in one burst per
 * step, resp. A fragments read one row block ahead; 13 = the 32x32x16
 * shape.  Any other value: SBO_E_INVAL.  (The timing diagnostics -- some
 * leave parts of the work out -- exist only in the diagnostic build
 * lib/libsbo_diag.so, never in this library.) */
#define SBO_OPT_KERNEL_VARIANT 5
/* SBO_OPT_SWEEP_GROUPS: workgroups of the persistent predictive sweep, each
 * walking one tile-balanced range of the tick's plan; 0 = default (one per
 * CU).  Results do not depend on it (bitwise). */
#define SBO_OPT_SWEEP_GROUPS 6
/* SBO_OPT_SKIP_BUDGET (B in [10, 60], default 20): the automatic K* cutoff
 * (SBO_OPT_TILE_SKIP = -1) keeps its worst-case error below 2^-B sf2 on any
 * variance and 2^-B sf2^(1/2) on any mean (2^-20 = 9.5e-7: under 10 % of the
 * 1e-5 contract; the measured effect at B = 18..27 is below the f32
 * rounding of the sweep itself).  Takes effect at the next sbo_fit /
 * sbo_append. */
#define SBO_OPT_SKIP_BUDGET 7
/* SBO_OPT_CHOLESKY (1 default | 2 | 0): the fit's factorization -- 1 the
 * library's blocked right-looking Cholesky (a one-workgroup kernel per
 * 128-column diagonal block, its own panel triangular solve, rocBLAS sgemm +
 * ssyrk for the trailing update with a look-ahead column), 2 the same with
 * rocBLAS strsm for the panel, 0 rocSOLVER spotrf.  Same f32 algorithm class
 * and the same NOT_SPD reporting (leading minor). */
#define SBO_OPT_CHOLESKY 8
/* SBO_OPT_INVERSE (1 default | 0): how the fit computes the f64 L^-1 of
 * SBO_OPT_INVERSE_BITS = 64 -- 1 the library's block recursion (rocSOLVER
 * dtrtri on diagonal blocks of <= 2048, the off-diagonal products as
 * panelled dgemms that leave out the zero half of each triangular factor:
 * n^3/3 flops), 0 rocsolver_dtrtri on the whole factor (its recursion
 * multiplies the triangles as full matrices: 2n^3/3).  Same algorithm
 * class; results agree to f64 rounding.  Takes effect at the next sbo_fit. */
#define SBO_OPT_INVERSE 9
/* SBO_OPT_JITTER_RETRIES (R in [0, 8], default 0): an sbo_fit whose
 * factorization fails (SBO_E_NOT_SPD: duplicate points with no noise, or a
 * kernel matrix singular in f32) is retried up to R times with
 * sf2 * 10^(r-7) added to the diagonal at retry r (1e-6 sf2, 1e-5 sf2, ...).
 * The jitter that succeeded becomes part of the noise term (appends and
 * exported state use it too) and sbo_get_jitter reports it; 0 keeps the
 * reference's behaviour of reporting the failure. */
#define SBO_OPT_JITTER_RETRIES 10
/* SBO_OPT_PRECISION (-1 auto default | 0 fast | 1 f64): the predictive
 * sweep's arithmetic.  0: the split-operand bf16 sweep (f32-accurate products,
 * f32 accumulation, A = sf2 L^-1 rounded to f32).  1: the precise sweep -- A
 * in f64 from the fit's f64 inverse, K* in f64, f64 MFMA
 * (v_mfma_f64_16x16x4_f64) and f64 sums; about 3-5x the fast sweep's time on
 * the same tiles.  -1: every sbo_fit (and an sbo_append once N grew by a
 * quarter since the last probe, SBO_OPT_REPROBE) sweeps a probe set -- a
 * 32 x 32 grid over the training box and up to 512 training locations
 * (sbo_get_probe) -- both ways and ticks with the precise sweep when the fast
 * sweep's variance error there, max |d var| / max var, exceeds 5e-6 (the 1e-5 contract over the largest whole-grid / probe ratio measured, 1.77;
 * 5e-6 * 2^(20 - B) for a looser SBO_OPT_SKIP_BUDGET B < 20):
 * dense data, where the variance is orders below sf2 and sf2 - |V|^2 cancels
 * (config/lpsc.yaml's own box at N = 16384).  The precise sweep's skip budget
 * is 2^-B times the smallest probe variance (SBO_OPT_SKIP_BUDGET = B).  Needs
 * SBO_OPT_INVERSE_BITS 64 and a fitted factor: an imported state always runs
 * the fast sweep.  Setting it on a fitted context takes effect at once. */
#define SBO_OPT_PRECISION 11
/* SBO_OPT_RESORT (percent, default 25; 0: never): sbo_append sorts each
 * batch only among itself (k-d), so scattered batches leave k-tiles whose
 * boxes span the domain and defeat the sweep's tile skipping.  Once the
 * points appended since the last sort exceed this share of the sorted ones,
 * the append re-sorts all points and refactors (a fit's cost, amortised over
 * the appends in between); otherwise it is the block Cholesky update.  The
 * posterior is the same either way (to f32 factorization rounding); caller
 * indices (sbo_get_order) are kept. */
#define SBO_OPT_RESORT 12
/* SBO_OPT_CHOL_RESERVE (CUs, default 0): the blocked Cholesky's trailing
 * updates (the look-ahead's second stream) run on a CU-masked stream that
 * leaves this many CUs free for the latency-bound chain of diagonal blocks and
 * panels.  Results do not depend on it (bitwise). */
#define SBO_OPT_CHOL_RESERVE 13
/* SBO_OPT_INV_OVERLAP (CUs, default 0: off): with the recursive f64 inverse,
 * its first half (the inverse of the factor's leading half and the product
 * below it: half the inverse's flops) starts as soon as the factor's left
 * half is final and runs beside the Cholesky's last steps, on a CU-masked
 * stream that leaves this many CUs to the factorization's latency-bound
 * chain.  Results do not depend on it (bitwise). */
#define SBO_OPT_INV_OVERLAP 14
/* SBO_OPT_CHOL_OUTER (columns, default 1024 since round 6; a multiple of
 * 128 in [128, 4096]): the blocked Cholesky's outer panel.  Each outer panel
 * is factored by the 128-column chain with its updates kept inside the
 * panel, and the rest of the trailing matrix takes one rank-1024 update per
 * outer panel; 128 is the one-level factorization (a rank-128 update per 128
 * columns).  1024 against 512: C4 fit -0.4 ms, the factor's backward error
 * 1.38e-7 -> 1.43e-7 (synthetic) and 8.7e-8 -> 9.5e-8 (lpsc box) at
 * N = 8192.  (Round 5 kept 512 when test_tile_skip_exact_and_bounded failed
 * at 1024; that leg compared a refit taking five inverse digits with the
 * first fit's dense sweep -- inverse drift, not the factor's -- and is fixed.) */
#define SBO_OPT_CHOL_OUTER 15
/* SBO_OPT_CHOL_DIAG (default 1): the blocked Cholesky's chain kernels -- the
 * 128 x 128 diagonal blocks (16-column panels) and the panel solves below
 * them -- with their inner updates on the matrix cores, left-looking (1: one
 * MFMA chain per block from every finished column, in registers) or
 * right-looking (2: each finished panel's update through LDS), or on the VALU
 * (0); the factor is bitwise the same. */
#define SBO_OPT_CHOL_DIAG 16
/* SBO_OPT_CHOL_GEMM (default 4): the blocked Cholesky's updates.  4 / 5: the
 * outer panels' two big updates (the look-ahead block column and the lower
 * trailing triangle, k = 512) as the int8-sliced GEMM of csrc/ozgemm.hip with
 * 4 / 5 base-256 digits per row (exact int32 digit products, one f64
 * combination per element, f32 out), from one pack of the panel per outer
 * step; the chain's small updates by rocBLAS.  C4 fit 41.3 -> 37.3 ms (5
 * digits: 39.0); the factor's backward error 1.64e-7 -> 1.38e-7 (synthetic,
 * N = 8192) and 2.51e-7 -> 8.7e-8 on the lpsc box against rocBLAS's f32
 * GEMMs.  0: rocBLAS sgemm / ssyrk; 1 / 2: the library's f32 matrix-core
 * kernel for the small trailing updates / every update (exact f32 products;
 * the factors agree to f32 rounding).  (3, the outer updates on the bf16
 * matrix cores with each operand split in three -- faster than rocBLAS, but
 * the factor's backward error 2.6x worse on the box -- exists only in the
 * diagnostic build; SBO_E_INVAL here.) */
#define SBO_OPT_CHOL_GEMM 17
/* SBO_OPT_INV_BASE (default 2048, in [1024, 8192], rounded down to a multiple
 * of 128) and SBO_OPT_INV_PANELS (default 16, in [1, 64]): the recursive f64
 * inverse's base-case size (rocSOLVER dtrtri on the diagonal blocks at
 * multiples of it) and the number of dgemm panels each of its products is cut
 * into (fewer panels: larger GEMMs, more multiplied zeros).  SBO_OPT_INV_LEAVES
 * (default 2): every base case up front -- with four or more full base cases
 * by doubling from 128-column blocks (one batched dtrtri, then two
 * strided-batched dgemms per product and level), else in one strided-batched
 * dtrtri (1: always the latter; 0: one call per base case inside the
 * recursion).  Tuning only; the inverse agrees to f64 rounding. */
#define SBO_OPT_INV_BASE 18
#define SBO_OPT_INV_PANELS 19
#define SBO_OPT_INV_LEAVES 20
/* SBO_OPT_REPROBE (percent, default 25; 0: every append): with
 * SBO_OPT_PRECISION -1, an sbo_append runs the precision probe again once N
 * has grown by this share since the last probe (every sbo_fit probes). */
#define SBO_OPT_REPROBE 21
/* SBO_OPT_PRECISE_KERNEL (3 default | 1 | 0): the precise sweep's arithmetic --
 * 1 A = sf2 L^-1 as five and K* as four balanced base-256 int8 digit slices, the 14
 * leading slice products on the int8 matrix cores (v_mfma_i32_16x16x64_i8,
 * exact int32 sums), combined in f64 per k-tile (an Ozaki-style sliced
 * product; predict_oz.hip), K*'s digits built in the sweep for every row
 * block that reads a k-tile; 3 the same products with K*'s digits read from a
 * table built once per (128-query block, k-tile) (the queries in chunks that
 * fit SBO_OPT_TABLE_MB; sigma bitwise kernel 1's); 0 every product and sum in
 * f64 on the f64 matrix cores (v_mfma_f64_16x16x4_f64; predict_f64.hip).  All
 * meet the 1e-5 contract where the fast sweep cannot (SBO_OPT_PRECISION). */
#define SBO_OPT_PRECISE_KERNEL 22
/* SBO_OPT_TABLE_MB (default 0 = automatic: 1/32 of the free device memory,
 * within [256 MiB, 8 GiB]): device memory budget, MiB, of the K* table
 * SBO_OPT_PRECISE_KERNEL 3 sweeps through (the queries run in chunks of as
 * many 128-query blocks as fit it; at least one). */
#define SBO_OPT_TABLE_MB 23
/* SBO_OPT_INV_OZ (default 6; 5, 4; 0: rocBLAS dgemm): the recursive f64
 * inverse's products at splits of 4096 and more (S = L21 A^-1, X21 = -C^-1 S;
 * N <= 32768)
 * as an f64 GEMM emulated on the int8 matrix cores -- each row / column cut
 * into that many base-256 digits under its own power of two, the digit
 * products summed exactly in int32, combined in f64 (csrc/ozgemm.hip).  Its
 * error is relative to a row's and a column's largest entries (2^-40 / 2^-48
 * of them for 5 / 6 digits), not to each product's: six digits move the
 * posterior by < 5e-7 against the dgemm fit, five by up to 4e-6 (not for the
 * precise regime).  With SBO_OPT_INV_OZ_ADAPT the value is the most digits a
 * fit uses.  The SBO_OPT_INV_OVERLAP fit keeps the dgemm products. */
#define SBO_OPT_INV_OZ 24
/* SBO_OPT_INV_CHECK (default 1; 0 off; 2 after every full inverse): the
 * fit's run-time accuracy guard of its f64 inverse X.  On 32 queries (a 4 x 4
 * lattice over the training box and 16 training locations) it forms V0 = X k
 * and one refinement against the f32 factor, V1 = V0 + X (k - L V0), in f64,
 * and takes err = max |(sf2 - |V0|^2) - (sf2 - |V1|^2)| / max (sf2 - |V1|^2):
 * the inverse's own share of the variance error, which the precision probe
 * cannot see (its two sweeps read the same inverse).  With 1 it runs after an
 * inverse whose products were int8-sliced (SBO_OPT_INV_OZ); when err exceeds
 * 5e-7 (a twentieth of the 1e-5 contract) the fit recomputes the inverse with
 * dgemm products and checks it again (sbo_get_inverse_check).  Runs on a
 * stream of its own beside the fit's operand packs. */
#define SBO_OPT_INV_CHECK 25
/* SBO_OPT_PLAN_BLOCK (0 = row-block-major; bi << 8 | bq): the item order of
 * the precise sweep's plans -- blocks of bi row blocks x bq query blocks, so
 * that the sweep workgroups of one XCD share the K* table pieces of a query
 * block in their L2 as well as the A tiles of a row block.  Results do not
 * depend on it (items are computed independently). */
#define SBO_OPT_PLAN_BLOCK 26
/* SBO_OPT_PROBE_SIZE (grid << 16 | train; default 32 << 16 | 512): the
 * precision probe's query set -- a grid x grid lattice over the training box
 * and `train` training locations (SBO_OPT_PRECISION); the next fit or append
 * probes again. */
#define SBO_OPT_PROBE_SIZE 27
/* SBO_OPT_INV_OZ_MIN (0 automatic, default; 2048, 4096, 8192): the smallest
 * split of the recursive inverse whose two products run as the int8-sliced
 * GEMM (SBO_OPT_INV_OZ); the levels below keep dgemm products.  Automatic:
 * 2048 for N >= 12288, else 4096. */
#define SBO_OPT_INV_OZ_MIN 28
/* SBO_OPT_INV_OZ_ADAPT (default 1; 0 off): the sliced inverse's digits per
 * fit from the guard's last readings (SBO_OPT_INV_CHECK must be on).  Both
 * grow ~256x per digit dropped (200-1000x measured), so a fit at d digits
 * with readings e (variance) and e_mu (mean) lets the next fit -- same
 * hyper-parameters, N and training bounding-box area within [0.8, 1.25] of
 * its -- take five digits when max(e, e_mu) 256^(d - 5) <= tol / 8 (never
 * four).  That fit must read both within tol / 8: otherwise it is redone at
 * SBO_OPT_INV_OZ digits (fired = 1) and the data keeps SBO_OPT_INV_OZ digits
 * from then on.  The first fit after sbo_create / sbo_warmup, after an
 * option change or a hyper-parameter change takes SBO_OPT_INV_OZ digits.
 * sbo_get_inverse_check's digits say which ran. */
#define SBO_OPT_INV_OZ_ADAPT 29
SBO_API sbo_status sbo_set_option(sbo_ctx *ctx, int option, int64_t value);

/* The last inverse check (SBO_OPT_INV_CHECK) of the current fit, on m = 31
 * guard queries (a 4 x 4 lattice over the training box, 15 training
 * locations).  ran = 1 if it ran; digits = the SBO_OPT_INV_OZ digits of the
 * checked inverse (0: dgemm).  Two readings, each the inverse's own share of
 * the posterior measured by one f64 refinement against the f32 factor:
 *   err       the variance's, max |d var| / max var (err_grid / err_train:
 *             over the lattice / the training locations, each normalised by
 *             its own largest variance; var_max the largest variance);
 *   err_mean  the mean's, max |d mu| / max |mu| (mean_max = max |mu|), from
 *             the residual y - m0 refined the same way (round 6: alpha, and
 *             so mu_ of src/safe_bayesian_optimization_node.cpp:642, comes
 *             from the same inverse).
 * fired = 1 if a reading exceeded its bound and the inverse was recomputed:
 * a six-digit (SBO_OPT_INV_OZ) inverse whose err or err_mean exceeds tol is
 * recomputed with dgemm products; a reduced-digit one (SBO_OPT_INV_OZ_ADAPT)
 * already above tol / 8 with SBO_OPT_INV_OZ digits, itself checked (and
 * recomputed with dgemm products if that one exceeds tol).  err_fallback /
 * err_mean_fallback: the readings of the recomputed inverse (-1 when none
 * was); kept_digits: the digits of the inverse the fit kept (0: dgemm); ms
 * the checks' device time.  Appends keep the fit's result (their new rows
 * are dgemm / dtrmv products). */
typedef struct sbo_inv_check {
    int32_t ran, fired, digits, m;
    double err, err_grid, err_train, err_fallback, tol, var_max, ms;
    double err_mean, mean_max, err_mean_fallback;
    int32_t kept_digits, reserved;
} sbo_inv_check;
SBO_API sbo_status sbo_get_inverse_check(const sbo_ctx *ctx, sbo_inv_check *out);

/* Release the fit-time and tick-time workspaces the context keeps between
 * calls for speed (the recursive inverse's scratch and the int8-sliced GEMM's
 * packed operands -- about 2.1 GB at N = 16384, 8.5 GB at 32768 -- the inverse
 * check's, the append re-sort's staging copy and the precise sweep's K* table,
 * up to SBO_OPT_TABLE_MB); they are allocated again on the next call that
 * needs them.  The fitted state (factor, inverse, operands) stays.  Waits for
 * the context's streams. */
SBO_API sbo_status sbo_trim(sbo_ctx *ctx);

/* Startup warm-up for the node's first map (no reference counterpart: the
 * node pays its first request_terrain_map, node.cpp:568-623, on a cold
 * process): fits n_cap synthetic points with `hyper` and the context's
 * options, then sweeps an m_cap-point raster grid with the fast and the
 * precise sweep, so that every code object a fit and a tick load (the
 * library's kernels, rocBLAS / rocSOLVER / Tensile) is loaded and the
 * workspaces are sized for fits of up to n_cap points and ticks of up to
 * m_cap queries.  The context is left unfitted (as after sbo_create); its
 * options are unchanged.  Synchronous. */
SBO_API sbo_status sbo_warmup(sbo_ctx *ctx, int64_t n_cap, int64_t m_cap, sbo_hyper hyper);

/* The sweep the ticks run (precise = 1: the f64 sweep) and the last probe
 * (SBO_OPT_PRECISION): the fast sweep's normwise variance error against the
 * precise one on the 32 x 32 probe grid and that grid's smallest and largest
 * variance (-1 when no probe ran).  SBO_E_STATE before a fit. */
SBO_API sbo_status sbo_get_precision(const sbo_ctx *ctx, int *precise, double *probe_err, double *probe_var_min,
                                     double *probe_var_max);

/* The last precision probe in detail (SBO_OPT_PRECISION): its query set is a
 * 32 x 32 grid over the training box (m_grid points) and m_train training
 * locations (every (n / m_train)-th stored point); err = the fast sweep's
 * max |d var| over both / the largest variance of both (the decision's
 * number, also sbo_get_precision's probe_err), err_grid / err_train = each
 * part's own max |d var| / its own largest variance.  err* = -1 when no
 * probe ran.  SBO_E_STATE before a fit. */
typedef struct sbo_probe {
    int32_t precise, m_grid, m_train, precise_kernel;   /* precise_kernel: SBO_OPT_PRECISE_KERNEL in effect */
    int64_t n_at_probe;
    double err, err_grid, err_train;
    double var_min, var_max, var_max_grid, var_max_train;
} sbo_probe;
SBO_API sbo_status sbo_get_probe(const sbo_ctx *ctx, sbo_probe *out);

/* The K* tile cutoff in effect (auto or fixed) and the norms it was derived from. */
SBO_API sbo_status sbo_get_skip(const sbo_ctx *ctx, int *cutoff_log2, double *max_row_l1, double *alpha_l1);

/* order[i] = the caller's index (position in the sbo_fit / sbo_append
 * inputs, appends numbered after the fit) of internal training row i. */
SBO_API sbo_status sbo_get_order(const sbo_ctx *ctx, int64_t *order);

/* Test accessor: the packed predictive operand A = sf2 * L^-1 unpacked into a
 * dense n x n ROW-major f32 host array (upper triangle left untouched). */
SBO_API sbo_status sbo_get_inverse(sbo_ctx *ctx, float *Linv);

/* Test accessor: the plan's per packed tile gain bounds, 8 floats per tile in
 * packed-tile order (row block I, k-tile t at tile_start(I) + t):
 * log2 of (16 max row 1-norm, spectral-norm bound, Frobenius norm, 0) of
 * A_It, then (16 max row 1-norm, spectral-norm bound) of its bf16 pieces A1
 * and A2 (-1000 for an all-zero matrix).  cap >= 8 * tiles. */
SBO_API sbo_status sbo_get_tile_bounds(sbo_ctx *ctx, float *bounds, int64_t cap);

/* Kernel timing (bench.py): when enabled, hipEvents are recorded on the
 * context's stream around every predictive-sweep and RBF-fill launch.
 * sbo_profile(ctx, 1) enables and resets; sbo_profile_read sums the elapsed
 * device time of the launches recorded so far (it synchronises on them). */
SBO_API sbo_status sbo_profile(sbo_ctx *ctx, int enable);
SBO_API sbo_status sbo_profile_read(sbo_ctx *ctx, double *predict_ms, int64_t *predict_launches,
                                    double *fill_ms, int64_t *fill_launches);
/* MFMA flops the predictive sweep actually executed since sbo_profile(ctx, 1)
 * (2*BM*BN*BK per multiplied tile; skipped exactly-zero tiles excluded). */
SBO_API sbo_status sbo_profile_work(sbo_ctx *ctx, double *predict_flops);
/* Matrix-core flops the predictive sweep issued since sbo_profile(ctx, 1):
 * 2*BM*BN*BK per MFMA product per multiplied tile -- six products per tile
 * for the split sweeps at full precision, three / one at the reduced
 * precision levels (variant 3), one for the f32 sweeps (variants 0, 1) and
 * the precise f64 sweep; tiles_by_level (may be NULL): the multiplied tiles
 * at six, three, one product(s). */
SBO_API sbo_status sbo_profile_mfma(sbo_ctx *ctx, double *mfma_flops, int64_t *tiles_by_level /* [3] or NULL */);
/* Diagnostic build only (libsbo_diag.so; the product returns zeros): with
 * SBO_OPT_KERNEL_VARIANT 39 (the default sweep with phase stamps,
 * s_memtime; never timed as the product) the summed cycles of every
 * sweep wave since the last call, cycles[0..11]: step top, half-step body,
 * item end, vmcnt wait, barrier, whole half-steps, body at six / three / one
 * product(s), half-steps at six / three / one product(s); then reset. */
SBO_API sbo_status sbo_debug_x3_stamps(sbo_ctx *ctx, double *cycles, int n);

#ifdef __cplusplus
}
#endif

#endif /* SBO_H_ */
