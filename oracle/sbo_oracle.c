/*
 * sbo_oracle.c -- CPU restatement of the safe-BO planning-tick hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity CHECKER for the MI355X
 * library (safe_bayesian_optimization_amd/csrc).  Only tests/, the smoke()
 * check in __graft_entry__.py and the cpu_baseline leg of bench.py may load
 * it.  The product path never links, calls or falls back to it.
 *
 * What it restates (file:line refer to /root/reference, the upstream
 * matthewyjiang/safe_bayesian_optimization snapshot):
 *
 *   GP mapper (a1-a4).  The reference does NOT contain the GP posterior: it
 *   receives mu/sigma from the external `terrain_mapping_node`
 *   (launch/safe_bayesian_optimization.launch.py:111-117) whose
 *   hyper-parameters are config/lpsc.yaml:35-37 (noise_level 0.1,
 *   length_scale 0.4, sigma_f 1.0).  The math contract restated here is
 *   SURVEY.md section 7:
 *       k(a,b) = sf2 * exp(-|a-b|^2 / (2 l^2)),  K = k(X,X) + sn2 I
 *       L = chol(K), alpha = K^-1 (y - m0)
 *       mu_q  = m0 + k_q^T alpha
 *       var_q = max(sf2 - |L^-1 k_q|^2, 0)          (latent variance)
 *   with sf2 = sigma_f^2 and sn2 = noise_level (a variance).
 *   PARITY vs the reference: UNPINNED (no source, no fixture exists); the
 *   restatement is pinned against scikit-learn's GaussianProcessRegressor
 *   (tests/golden/make_golden.py) as an independent implementation.
 *
 *   ComputeConfidenceIntervals / UpdateSafeSet
 *       src/safe_bayesian_optimization_node.cpp:409-416
 *   FindSafetyContourIndices   :418-497 (raster + cv::findContours + index map)
 *   GetNextSubgoal             :499-550
 *
 *   cv::findContours(RETR_EXTERNAL, CHAIN_APPROX_NONE) is a third-party
 *   dependency absent from /root/reference (OpenCV, version unpinned by
 *   CMakeLists.txt:28; Ubuntu 22.04/ROS Humble ships 4.5.4).  It is restated
 *   from OpenCV 4.5.x's published Suzuki-Abe border follower (legacy C
 *   implementation: 1-px zero padding, raster scan, external-only starts,
 *   counter-clockwise trace, every traversed pixel emitted, contours returned
 *   in reverse discovery order).  Contour ORDER is parity-unpinned.
 *
 * Compile with -ffp-contract=off: the reference's Eigen arithmetic is plain
 * IEEE double without fused multiply-add on x86-64.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <limits.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_EXPORT __attribute__((visibility("default")))

ORC_EXPORT void orc_set_threads(int n)
{
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

ORC_EXPORT int orc_get_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* ------------------------------------------------------------------------ */
/* a1: RBF kernel matrix (column-major, lda = n).                            */
/* ------------------------------------------------------------------------ */
ORC_EXPORT void orc_rbf_fill(const double *x, const double *y, int64_t n,
                             double ell, double sf2, double sn2, double *K)
{
    const double inv2l2 = 1.0 / (2.0 * ell * ell);
#pragma omp parallel for schedule(static)
    for (int64_t j = 0; j < n; ++j) {
        for (int64_t i = 0; i < n; ++i) {
            const double dx = x[i] - x[j], dy = y[i] - y[j];
            double v = sf2 * exp(-(dx * dx + dy * dy) * inv2l2);
            if (i == j) v += sn2;
            K[i + j * n] = v;
        }
    }
}

/* fp32 coordinates in, fp64 values out: the elementwise reference for the
 * device fill (the test rounds it to f32 and compares in ulps). */
ORC_EXPORT void orc_rbf_fill_f32in(const float *x, const float *y, int64_t n,
                                   double ell, double sf2, double sn2, double *K)
{
    const double inv2l2 = 1.0 / (2.0 * ell * ell);
#pragma omp parallel for schedule(static)
    for (int64_t j = 0; j < n; ++j) {
        for (int64_t i = 0; i < n; ++i) {
            const double dx = (double)x[i] - (double)x[j];
            const double dy = (double)y[i] - (double)y[j];
            double v = sf2 * exp(-(dx * dx + dy * dy) * inv2l2);
            if (i == j) v += sn2;
            K[i + j * n] = v;
        }
    }
}

/* The device fill's own f32 formulation (dx, dy, d2 = fmaf(dy,dy,dx*dx),
 * arg = c*d2 with c = -1/(2 l^2) in f32, sf2*expf(arg) [+ sn2]), so that the
 * only difference left against the device is the expf implementation
 * (SURVEY.md 8(c) stage 1: <= 2 ulp). */
ORC_EXPORT void orc_rbf_fill_f32(const float *x, const float *y, int64_t n,
                                 float ell, float sf2, float sn2, float *K)
{
    const float c = -1.0f / (2.0f * ell * ell);
#pragma omp parallel for schedule(static)
    for (int64_t j = 0; j < n; ++j) {
        for (int64_t i = 0; i < n; ++i) {
            const float dx = x[i] - x[j], dy = y[i] - y[j];
            float v = sf2 * expf(c * fmaf(dy, dy, dx * dx));
            if (i == j) v += sn2;
            K[i + j * n] = v;
        }
    }
}

/* Cross kernel K*^T (n x m, column-major, f32) for the bench's dense CPU
 * comparator (bench.py cpu_baseline, oracle.BlasPredictor): column q holds
 * sf2 * exp(-|x_i - q|^2 / (2 l^2)) over the n training points, one OpenMP
 * thread per block of query columns -- the Eigen-class path builds K* on
 * every host core before its triangular solve.  Same f32 formulation as
 * orc_rbf_fill_f32. */
ORC_EXPORT void orc_cross_kernel_f32(const float *x, const float *y, int64_t n, const float *qx,
                                     const float *qy, int64_t m, float ell, float sf2, float *Ks)
{
    const float c = -1.0f / (2.0f * ell * ell);
#pragma omp parallel for schedule(static)
    for (int64_t q = 0; q < m; ++q) {
        float *col = Ks + q * n;
        const float a = qx[q], b = qy[q];
        for (int64_t i = 0; i < n; ++i) {
            const float dx = x[i] - a, dy = y[i] - b;
            col[i] = sf2 * expf(c * fmaf(dy, dy, dx * dx));
        }
    }
}

/* ------------------------------------------------------------------------ */
/* a2: blocked right-looking Cholesky, lower, column-major, in place.        */
/* Returns 0 on success, k+1 if the leading minor of order k+1 is not SPD.  */
/* ------------------------------------------------------------------------ */
#define ORC_NB 64

static int64_t chol_unblocked(double *A, int64_t n, int64_t k0, int64_t kb)
{
    for (int64_t k = k0; k < k0 + kb; ++k) {
        double d = A[k + k * n];
        for (int64_t p = k0; p < k; ++p) d -= A[k + p * n] * A[k + p * n];
        if (!(d > 0.0)) return k + 1;
        d = sqrt(d);
        A[k + k * n] = d;
        for (int64_t i = k + 1; i < k0 + kb; ++i) {
            double s = A[i + k * n];
            for (int64_t p = k0; p < k; ++p) s -= A[i + p * n] * A[k + p * n];
            A[i + k * n] = s / d;
        }
    }
    return 0;
}

ORC_EXPORT int64_t orc_cholesky(double *A, int64_t n)
{
    for (int64_t k0 = 0; k0 < n; k0 += ORC_NB) {
        const int64_t kb = (n - k0 < ORC_NB) ? n - k0 : ORC_NB;
        const int64_t info = chol_unblocked(A, n, k0, kb);
        if (info) return info;
        /* panel: A[i, k0:k0+kb] <- A[i, k0:k0+kb] * L11^-T for i >= k0+kb */
#pragma omp parallel for schedule(static)
        for (int64_t i = k0 + kb; i < n; ++i) {
            for (int64_t k = k0; k < k0 + kb; ++k) {
                double s = A[i + k * n];
                for (int64_t p = k0; p < k; ++p) s -= A[i + p * n] * A[k + p * n];
                A[i + k * n] = s / A[k + k * n];
            }
        }
        /* trailing update of the lower triangle, column by column */
#pragma omp parallel for schedule(dynamic, 16)
        for (int64_t j = k0 + kb; j < n; ++j) {
            for (int64_t p = k0; p < k0 + kb; ++p) {
                const double ajp = A[j + p * n];
                const double *colp = A + p * n;
                double *colj = A + j * n;
                for (int64_t i = j; i < n; ++i) colj[i] -= colp[i] * ajp;
            }
        }
    }
    return 0;
}

/* Solve (L L^T) x = b for one right-hand side (L column-major lower). */
ORC_EXPORT void orc_chol_solve(const double *L, int64_t n, const double *b, double *x)
{
    for (int64_t i = 0; i < n; ++i) x[i] = b[i];
    for (int64_t j = 0; j < n; ++j) {           /* forward: L z = b */
        x[j] /= L[j + j * n];
        const double xj = x[j];
        for (int64_t i = j + 1; i < n; ++i) x[i] -= L[i + j * n] * xj;
    }
    for (int64_t i = n - 1; i >= 0; --i) {      /* backward: L^T a = z */
        double s = x[i];
        for (int64_t k = i + 1; k < n; ++k) s -= L[k + i * n] * x[k];
        x[i] = s / L[i + i * n];
    }
}

/* ------------------------------------------------------------------------ */
/* a3+a4: posterior mean / latent variance for a block of queries.          */
/* Instantiated for double (parity) and float (CPU baseline timing).        */
/* ------------------------------------------------------------------------ */
#define ORC_QB 64

#define ORC_DEFINE_PREDICT(REAL, EXPF, SQRTF, NAME)                                   \
ORC_EXPORT void NAME(const REAL *L, const REAL *alpha, const REAL *X, const REAL *Y, \
                     int64_t n, double ell, double sf2_d, double m0_d,               \
                     const REAL *qx, const REAL *qy, int64_t m,                      \
                     REAL *mu, REAL *var)                                            \
{                                                                                    \
    const REAL inv2l2 = (REAL)(1.0 / (2.0 * ell * ell));                             \
    const REAL sf2 = (REAL)sf2_d, m0 = (REAL)m0_d;                                   \
    /* row-major copy of the lower factor for unit-stride row access */              \
    REAL *Lr = (REAL *)malloc(sizeof(REAL) * (size_t)n * (size_t)n);                 \
    _Pragma("omp parallel for schedule(static)")                                     \
    for (int64_t i = 0; i < n; ++i)                                                  \
        for (int64_t j = 0; j <= i; ++j) Lr[i * n + j] = L[i + j * n];               \
    const int64_t nqb = (m + ORC_QB - 1) / ORC_QB;                                   \
    _Pragma("omp parallel")                                                          \
    {                                                                                \
        REAL *V = (REAL *)malloc(sizeof(REAL) * (size_t)n * ORC_QB);                 \
        _Pragma("omp for schedule(dynamic, 1)")                                      \
        for (int64_t b = 0; b < nqb; ++b) {                                          \
            const int64_t q0 = b * ORC_QB;                                           \
            const int64_t qn = (m - q0 < ORC_QB) ? m - q0 : ORC_QB;                  \
            /* V[i][c] = k(x_i, q_c) */                                              \
            for (int64_t i = 0; i < n; ++i)                                          \
                for (int64_t c = 0; c < ORC_QB; ++c) {                               \
                    const int64_t q = q0 + (c < qn ? c : 0);                         \
                    const REAL dx = X[i] - qx[q], dy = Y[i] - qy[q];                 \
                    V[i * ORC_QB + c] = sf2 * EXPF(-(dx * dx + dy * dy) * inv2l2);   \
                }                                                                    \
            REAL acc_mu[ORC_QB];                                                     \
            for (int64_t c = 0; c < ORC_QB; ++c) acc_mu[c] = 0;                      \
            for (int64_t i = 0; i < n; ++i) {                                        \
                const REAL a = alpha[i];                                             \
                for (int64_t c = 0; c < ORC_QB; ++c) acc_mu[c] += a * V[i * ORC_QB + c]; \
            }                                                                        \
            /* blocked forward substitution  L V = K*^T */                           \
            for (int64_t i0 = 0; i0 < n; i0 += ORC_NB) {                             \
                const int64_t ie = (i0 + ORC_NB < n) ? i0 + ORC_NB : n;              \
                for (int64_t i = i0; i < ie; ++i) {                                  \
                    REAL *vi = V + i * ORC_QB;                                       \
                    const REAL *li = Lr + i * n;                                     \
                    for (int64_t j = 0; j < i; ++j) {                                \
                        const REAL l = li[j];                                        \
                        const REAL *vj = V + j * ORC_QB;                             \
                        for (int64_t c = 0; c < ORC_QB; ++c) vi[c] -= l * vj[c];     \
                    }                                                                \
                    const REAL d = li[i];                                            \
                    for (int64_t c = 0; c < ORC_QB; ++c) vi[c] /= d;                 \
                }                                                                    \
            }                                                                        \
            for (int64_t c = 0; c < qn; ++c) {                                       \
                REAL s = 0;                                                          \
                for (int64_t i = 0; i < n; ++i) s += V[i * ORC_QB + c] * V[i * ORC_QB + c]; \
                REAL v = sf2 - s;                                                    \
                var[q0 + c] = v > 0 ? v : 0;                                         \
                mu[q0 + c] = m0 + acc_mu[c];                                         \
            }                                                                        \
        }                                                                            \
        free(V);                                                                     \
    }                                                                                \
    free(Lr);                                                                        \
}

ORC_DEFINE_PREDICT(double, exp, sqrt, orc_predict)
ORC_DEFINE_PREDICT(float, expf, sqrtf, orc_predict_f32)

/* The posterior mean alone (a3, the `values` the node copies into mu_,
 * src/safe_bayesian_optimization_node.cpp:642): mu_q = m0 + sum_i alpha_i
 * sf2 exp(-|x_i - q|^2 / (2 l^2)), in f64, the same terms and order as
 * orc_predict's acc_mu -- O(n) per query, so the tests can hold the mean of a
 * whole 10^6-point grid to the oracle (tests/test_gpu_precision.py). */
ORC_EXPORT void orc_predict_mean(const double *alpha, const double *X, const double *Y, int64_t n, double ell,
                                 double sf2, double m0, const double *qx, const double *qy, int64_t m, double *mu)
{
    const double inv2l2 = 1.0 / (2.0 * ell * ell);
    _Pragma("omp parallel for schedule(static, 256)")
    for (int64_t q = 0; q < m; ++q) {
        double acc = 0.0;
        for (int64_t i = 0; i < n; ++i) {
            const double dx = X[i] - qx[q], dy = Y[i] - qy[q];
            acc += alpha[i] * (sf2 * exp(-(dx * dx + dy * dy) * inv2l2));
        }
        mu[q] = m0 + acc;
    }
}

/* ------------------------------------------------------------------------ */
/* a6+a7: ComputeConfidenceIntervals + UpdateSafeSet                          */
/*   src/safe_bayesian_optimization_node.cpp:411-416 and :409               */
/*   confidence = beta * std;  Q(:,0) = mu - confidence;  Q(:,1) = mu + c   */
/*   S = Q(:,0) > f_min   (strict)                                           */
/* ------------------------------------------------------------------------ */
ORC_EXPORT void orc_compute_sets(const double *mu, const double *sd, int64_t m,
                                 double beta, double f_min,
                                 double *lo, double *hi, uint8_t *safe)
{
    for (int64_t i = 0; i < m; ++i) {
        const double c = beta * sd[i];
        lo[i] = mu[i] - c;
        hi[i] = mu[i] + c;
        safe[i] = lo[i] > f_min ? 1 : 0;
    }
}

/* a10: masked argmax, highest score, lowest index on ties, NaN never wins.
 * Returns the index or -1 when nothing is eligible. */
ORC_EXPORT int64_t orc_argmax(const double *score, const uint8_t *mask, int64_t m, double *val)
{
    int64_t best = -1;
    double bv = 0.0;
    for (int64_t i = 0; i < m; ++i) {
        if (mask && !mask[i]) continue;
        const double s = score[i];
        if (s != s) continue;
        if (best < 0 || s > bv) { best = i; bv = s; }
    }
    if (val) *val = bv;
    return best;
}

/* ------------------------------------------------------------------------ */
/* cv::findContours(img, RETR_EXTERNAL, CHAIN_APPROX_NONE), OpenCV 4.5.x.   */
/* img: h rows x w cols, row-major u8, nonzero = foreground.                */
/* Output: pts = (x,y) pairs, start[c] = first point of contour c,           */
/* start[nc] = total points.  Contours are emitted in OpenCV's return order */
/* (reverse discovery).  Returns the number of contours, or -1 if a          */
/* capacity is exceeded.                                                     */
/* ------------------------------------------------------------------------ */
static const int orc_dx8[8] = {1, 1, 0, -1, -1, -1, 0, 1};
static const int orc_dy8[8] = {0, -1, -1, -1, 0, 1, 1, 1};

ORC_EXPORT int64_t orc_find_contours_external(const uint8_t *img, int w, int h,
                                              int32_t *pts, int64_t pts_cap,
                                              int64_t *start, int64_t contours_cap)
{
    if (w <= 0 || h <= 0) return 0;
    const int64_t W = (int64_t)w + 2, H = (int64_t)h + 2;
    signed char *im = (signed char *)calloc((size_t)(W * H), 1);
    for (int64_t y = 0; y < h; ++y)
        for (int64_t x = 0; x < w; ++x)
            im[(y + 1) * W + (x + 1)] = img[y * w + x] ? 1 : 0;

    /* discovery-order scratch */
    int64_t dcap = 1024, dn = 0, pn = 0, pcap = 4096;
    int64_t *dstart = (int64_t *)malloc(sizeof(int64_t) * (size_t)(dcap + 1));
    int32_t *dp = (int32_t *)malloc(sizeof(int32_t) * 2 * (size_t)pcap);

#define ORC_EMIT(px, py)                                                          \
    do {                                                                          \
        if (pn == pcap) { pcap *= 2; dp = (int32_t *)realloc(dp, sizeof(int32_t) * 2 * (size_t)pcap); } \
        dp[2 * pn] = (int32_t)((px) - 1); dp[2 * pn + 1] = (int32_t)((py) - 1); ++pn; \
    } while (0)

    for (int64_t y = 1; y < H - 1; ++y) {
        int prev = 0;
        int64_t lnbd_x = 0;                      /* last marked border pixel on this row */
        for (int64_t x = 1; x < W - 1; ++x) {
            const int p = im[y * W + x];
            if (p == prev) continue;
            if (prev == 0 && p == 1 && !(im[y * W + lnbd_x] > 0)) {
                /* new outer border (external mode: not inside another outer border) */
                if (dn == dcap) { dcap *= 2; dstart = (int64_t *)realloc(dstart, sizeof(int64_t) * (size_t)(dcap + 1)); }
                dstart[dn++] = pn;
                lnbd_x = x;
                const int64_t i0 = y * W + x;
                int s = 4;
                int64_t i1 = i0;
                do {
                    s = (s - 1) & 7;
                    i1 = i0 + orc_dx8[s] + orc_dy8[s] * W;
                } while (im[i1] == 0 && s != 4);
                if (s == 4) {                    /* isolated pixel */
                    im[i0] = (signed char)-126;
                    ORC_EMIT(x, y);
                } else {
                    int64_t i3 = i0, i4 = i0;
                    int64_t cx = x, cy = y;
                    for (;;) {
                        const int s_end = s;
                        int t = s;
                        while (t < 15) {         /* counter-clockwise search after s */
                            ++t;
                            i4 = i3 + orc_dx8[t & 7] + orc_dy8[t & 7] * W;
                            if (im[i4] != 0) break;
                        }
                        s = t & 7;
                        if ((unsigned)(s - 1) < (unsigned)s_end) im[i3] = (signed char)-126;
                        else if (im[i3] == 1) im[i3] = 2;
                        ORC_EMIT(cx, cy);
                        cx += orc_dx8[s];
                        cy += orc_dy8[s];
                        if (i4 == i0 && i3 == i1) break;
                        i3 = i4;
                        s = (s + 4) & 7;
                    }
                }
                prev = im[y * W + x];            /* scanner resumes after the start pixel */
                continue;
            }
            prev = p;
            if (p & -2) lnbd_x = x;              /* marked border pixel (2 or negative) */
        }
    }
    dstart[dn] = pn;
#undef ORC_EMIT

    int64_t ret = dn;
    if (dn > contours_cap || pn > pts_cap) {
        ret = -1;
    } else {
        /* reverse discovery order, as the contour tree is built head-first */
        int64_t o = 0;
        for (int64_t c = 0; c < dn; ++c) {
            const int64_t src = dn - 1 - c;
            start[c] = o;
            for (int64_t k = dstart[src]; k < dstart[src + 1]; ++k) {
                pts[2 * o] = dp[2 * k];
                pts[2 * o + 1] = dp[2 * k + 1];
                ++o;
            }
        }
        start[dn] = o;
    }
    free(dp);
    free(dstart);
    free(im);
    return ret;
}

/* static_cast<int>(double) as executed on x86-64 (cvttsd2si): values that are
 * NaN or outside the int range come out as INT_MIN. */
static int orc_trunc_int(double v)
{
    if (!(v > -2147483649.0 && v < 2147483648.0)) return INT_MIN;
    return (int)v;
}

/* FindSafetyContourIndices, src/safe_bayesian_optimization_node.cpp:418-497.
 * Dx, Dy: grid coordinates (D_ columns, f64).  Returns the number of frontier
 * indices written to out (duplicates kept), or -1 if out_cap is too small. */
ORC_EXPORT int64_t orc_find_safety_contour_indices(const double *Dx, const double *Dy,
                                                   const uint8_t *safe, int64_t m,
                                                   int width, int height,
                                                   int32_t *out, int64_t out_cap)
{
    if (m <= 0 || width <= 0 || height <= 0) return 0;
    double mnx = Dx[0], mxx = Dx[0], mny = Dy[0], mxy = Dy[0];
    for (int64_t i = 1; i < m; ++i) {
        if (Dx[i] < mnx) mnx = Dx[i];
        if (Dx[i] > mxx) mxx = Dx[i];
        if (Dy[i] < mny) mny = Dy[i];
        if (Dy[i] > mxy) mxy = Dy[i];
    }
    const int min_x = orc_trunc_int(mnx), max_x = orc_trunc_int(mxx);
    const int min_y = orc_trunc_int(mny), max_y = orc_trunc_int(mxy);
    const int64_t npx = (int64_t)width * height;
    uint8_t *img = (uint8_t *)calloc((size_t)npx, 1);
    int32_t *owner = (int32_t *)malloc(sizeof(int32_t) * (size_t)npx);
    for (int64_t k = 0; k < npx; ++k) owner[k] = -1;
    for (int64_t i = 0; i < m; ++i) {
        const int x = orc_trunc_int((Dx[i] - min_x) / (double)(max_x - min_x) * width);
        const int y = orc_trunc_int((Dy[i] - min_y) / (double)(max_y - min_y) * height);
        if (x >= 0 && x < width && y >= 0 && y < height) {
            img[(int64_t)y * width + x] = safe[i] ? 255 : 0;   /* last writer wins */
            owner[(int64_t)y * width + x] = (int32_t)i;        /* coord_to_index[x][y] = i */
        }
    }
    const int64_t pcap = 8 * npx + 16, ccap = npx + 1;
    int32_t *pts = (int32_t *)malloc(sizeof(int32_t) * 2 * (size_t)pcap);
    int64_t *st = (int64_t *)malloc(sizeof(int64_t) * (size_t)(ccap + 1));
    const int64_t nc = orc_find_contours_external(img, width, height, pts, pcap, st, ccap);
    int64_t cnt = 0;
    if (nc > 0) {
        for (int64_t k = 0; k < st[nc]; ++k) {
            const int32_t px = pts[2 * k], py = pts[2 * k + 1];
            const int32_t idx = owner[(int64_t)py * width + px];
            if (idx < 0) continue;
            if (cnt >= out_cap) { cnt = -1; break; }
            out[cnt++] = idx;
        }
    }
    free(st);
    free(pts);
    free(owner);
    free(img);
    return cnt;
}

/* GetNextSubgoal, src/safe_bayesian_optimization_node.cpp:499-550. */
typedef struct { double d; size_t i; } orc_pair;

static int orc_pair_cmp(const void *a, const void *b)
{
    const orc_pair *x = (const orc_pair *)a, *y = (const orc_pair *)b;
    if (x->d < y->d) return -1;
    if (x->d > y->d) return 1;
    if (x->i < y->i) return -1;
    if (x->i > y->i) return 1;
    return 0;
}

ORC_EXPORT int64_t orc_next_subgoal(const double *Dx, const double *Dy,
                                    const double *lo, const double *hi, const uint8_t *safe,
                                    int64_t m, int width, int height, double gx, double gy)
{
    if (m <= 0) return -1;
    int64_t cap = 8 * (int64_t)width * height + 16;
    int32_t *F = (int32_t *)malloc(sizeof(int32_t) * (size_t)cap);
    const int64_t nf = orc_find_safety_contour_indices(Dx, Dy, safe, m, width, height, F, cap);
    if (nf <= 0) { free(F); return -1; }
    orc_pair *pairs = (orc_pair *)malloc(sizeof(orc_pair) * (size_t)nf);
    double *wid = (double *)malloc(sizeof(double) * (size_t)nf);
    for (int64_t i = 0; i < nf; ++i) {
        const int32_t idx = F[i];
        wid[i] = hi[idx] - lo[idx];
        const double dx = Dx[idx] - gx, dy = Dy[idx] - gy;
        pairs[i].d = sqrt(dx * dx + dy * dy);
        pairs[i].i = (size_t)i;
    }
    qsort(pairs, (size_t)nf, sizeof(orc_pair), orc_pair_cmp);
    size_t top = (size_t)nf / 4;
    if (top < 1) top = 1;
    double best_w = -1.0;
    int64_t best = -1;
    for (size_t t = 0; t < top; ++t) {
        const size_t fi = pairs[t].i;
        if (wid[fi] > best_w) { best_w = wid[fi]; best = (int64_t)fi; }
    }
    /* Deliberate divergence, "given the builder's restatement": when no
     * frontier width exceeds -1 (every width NaN, e.g. a NaN sigma), the
     * node's best_index stays -1 and it reads frontier_indices[-1]
     * (node.cpp:537-549, undefined behaviour); the restatement returns -1
     * ("no subgoal", as node.cpp:503-506 does for an empty frontier). */
    const int64_t r = best >= 0 ? F[best] : -1;
    free(wid);
    free(pairs);
    free(F);
    return r;
}
