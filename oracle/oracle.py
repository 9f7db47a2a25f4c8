"""ctypes front-end for the CPU oracle (``liboracle.so``).

TEST INFRASTRUCTURE ONLY: the parity checker for the MI355X library.  Only
``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` import this module.  The product package never imports it.

Every function restates a reference code path (see ``sbo_oracle.c`` for the
file:line citations) or the GP math contract of SURVEY.md section 7.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.environ.get("ORC_LIB") or os.path.join(_HERE, "liboracle.so")   # ORC_LIB: sanitizer build
_lib = None

_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
_i64 = ctypes.c_int64
_dbl = ctypes.c_double


def build() -> str:
    """Compile liboracle.so in place (gcc only)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.orc_set_threads.argtypes = [ctypes.c_int]
        L.orc_get_threads.restype = ctypes.c_int
        L.orc_rbf_fill.argtypes = [_f64p, _f64p, _i64, _dbl, _dbl, _dbl, _f64p]
        L.orc_rbf_fill_f32in.argtypes = [_f32p, _f32p, _i64, _dbl, _dbl, _dbl, _f64p]
        L.orc_rbf_fill_f32.argtypes = [_f32p, _f32p, _i64, ctypes.c_float, ctypes.c_float,
                                       ctypes.c_float, _f32p]
        L.orc_cross_kernel_f32.argtypes = [_f32p, _f32p, _i64, _f32p, _f32p, _i64, ctypes.c_float,
                                           ctypes.c_float, ctypes.c_void_p]
        L.orc_cholesky.argtypes = [_f64p, _i64]
        L.orc_cholesky.restype = _i64
        L.orc_chol_solve.argtypes = [_f64p, _i64, _f64p, _f64p]
        L.orc_predict.argtypes = [_f64p, _f64p, _f64p, _f64p, _i64, _dbl, _dbl, _dbl,
                                  _f64p, _f64p, _i64, _f64p, _f64p]
        L.orc_predict_f32.argtypes = [_f32p, _f32p, _f32p, _f32p, _i64, _dbl, _dbl, _dbl,
                                      _f32p, _f32p, _i64, _f32p, _f32p]
        L.orc_predict_mean.argtypes = [_f64p, _f64p, _f64p, _i64, _dbl, _dbl, _dbl, _f64p, _f64p, _i64, _f64p]
        L.orc_compute_sets.argtypes = [_f64p, _f64p, _i64, _dbl, _dbl, _f64p, _f64p, _u8p]
        L.orc_argmax.argtypes = [_f64p, ctypes.c_void_p, _i64, ctypes.POINTER(_dbl)]
        L.orc_argmax.restype = _i64
        L.orc_find_contours_external.argtypes = [_u8p, ctypes.c_int, ctypes.c_int,
                                                 _i32p, _i64, _i64p, _i64]
        L.orc_find_contours_external.restype = _i64
        L.orc_find_safety_contour_indices.argtypes = [_f64p, _f64p, _u8p, _i64,
                                                      ctypes.c_int, ctypes.c_int, _i32p, _i64]
        L.orc_find_safety_contour_indices.restype = _i64
        L.orc_next_subgoal.argtypes = [_f64p, _f64p, _f64p, _f64p, _u8p, _i64,
                                       ctypes.c_int, ctypes.c_int, _dbl, _dbl]
        L.orc_next_subgoal.restype = _i64
        _lib = L
    return _lib


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def set_threads(n: int) -> None:
    lib().orc_set_threads(int(n))


def get_threads() -> int:
    return int(lib().orc_get_threads())


# ---------------------------------------------------------------- GP (a1-a4)
def rbf_fill(x, y, ell=0.4, sf2=1.0, sn2=0.1):
    """K = sf2 exp(-d^2/2l^2) + sn2 I, column-major (returned as K[j, i])."""
    x = _c(x, np.float64); y = _c(y, np.float64)
    n = x.size
    K = np.empty(n * n, np.float64)
    lib().orc_rbf_fill(x, y, n, ell, sf2, sn2, K)
    return K.reshape(n, n)  # symmetric: row/col major identical


def rbf_fill_f32in(x, y, ell=0.4, sf2=1.0, sn2=0.1):
    x = _c(x, np.float32); y = _c(y, np.float32)
    n = x.size
    K = np.empty(n * n, np.float64)
    lib().orc_rbf_fill_f32in(x, y, n, ell, sf2, sn2, K)
    return K.reshape(n, n)


def rbf_fill_f32(x, y, ell=0.4, sf2=1.0, sn2=0.1):
    """The device fill's f32 formulation (column-major == row-major, symmetric)."""
    x = _c(x, np.float32); y = _c(y, np.float32)
    n = x.size
    K = np.empty(n * n, np.float32)
    lib().orc_rbf_fill_f32(x, y, n, ell, sf2, sn2, K)
    return K.reshape(n, n)


def cholesky(K):
    """Lower Cholesky factor (column-major buffer returned as an (n, n) array
    A with A[j, i] = L[i, j]; use ``lower_from_colmajor`` for L)."""
    n = K.shape[0]
    A = np.array(K, dtype=np.float64, order="C").reshape(-1).copy()
    info = lib().orc_cholesky(A, n)
    if info:
        raise np.linalg.LinAlgError(f"oracle cholesky: leading minor {info} not SPD")
    return A.reshape(n, n)


def lower_from_colmajor(A):
    """(n, n) array holding a column-major buffer -> dense lower L (row-major)."""
    return np.tril(A.T)


def colmajor_from_lower(L):
    return np.ascontiguousarray(np.asarray(L, np.float64).T)


def chol_solve(Acm, b):
    n = Acm.shape[0]
    out = np.empty(n, np.float64)
    lib().orc_chol_solve(np.ascontiguousarray(Acm, np.float64).reshape(-1), n, _c(b, np.float64), out)
    return out


def fit(x, y, obs, ell=0.4, sf2=1.0, sn2=0.1, m0=0.0):
    """fp64 GP fit: returns (Lcm, alpha) with Lcm column-major (see cholesky)."""
    K = rbf_fill(x, y, ell, sf2, sn2)
    Lcm = cholesky(K)
    alpha = chol_solve(Lcm, _c(obs, np.float64) - m0)
    return Lcm, alpha


def predict(Lcm, alpha, x, y, qx, qy, ell=0.4, sf2=1.0, m0=0.0):
    """fp64 posterior mean and latent variance at the query points."""
    n = alpha.size
    qx = _c(qx, np.float64); qy = _c(qy, np.float64)
    m = qx.size
    mu = np.empty(m, np.float64); var = np.empty(m, np.float64)
    lib().orc_predict(np.ascontiguousarray(Lcm, np.float64).reshape(-1), _c(alpha, np.float64),
                      _c(x, np.float64), _c(y, np.float64), n, ell, sf2, m0, qx, qy, m, mu, var)
    return mu, var


def predict_mean(alpha, x, y, qx, qy, ell=0.4, sf2=1.0, m0=0.0):
    """fp64 posterior mean alone (O(n) per query: whole grids)."""
    qx = _c(qx, np.float64); qy = _c(qy, np.float64)
    mu = np.empty(qx.size, np.float64)
    lib().orc_predict_mean(_c(alpha, np.float64), _c(x, np.float64), _c(y, np.float64), alpha.size, ell, sf2, m0,
                           qx, qy, qx.size, mu)
    return mu


def predict_f32(Lcm, alpha, x, y, qx, qy, ell=0.4, sf2=1.0, m0=0.0):
    n = alpha.size
    qx = _c(qx, np.float32); qy = _c(qy, np.float32)
    m = qx.size
    mu = np.empty(m, np.float32); var = np.empty(m, np.float32)
    lib().orc_predict_f32(np.ascontiguousarray(Lcm, np.float32).reshape(-1), _c(alpha, np.float32),
                          _c(x, np.float32), _c(y, np.float32), n, ell, sf2, m0, qx, qy, m, mu, var)
    return mu, var


# ------------------------------------------------------- acquisition (a6-a10)
def compute_sets(mu, sd, beta, f_min):
    """ComputeConfidenceIntervals + UpdateSafeSet (node.cpp:409-416)."""
    mu = _c(mu, np.float64); sd = _c(sd, np.float64)
    m = mu.size
    lo = np.empty(m, np.float64); hi = np.empty(m, np.float64); s = np.empty(m, np.uint8)
    lib().orc_compute_sets(mu, sd, m, float(beta), float(f_min), lo, hi, s)
    return lo, hi, s


def argmax(score, mask=None):
    score = _c(score, np.float64)
    val = _dbl(0.0)
    if mask is not None:
        mask = _c(mask, np.uint8)
        ptr = mask.ctypes.data_as(ctypes.c_void_p)
    else:
        ptr = None
    idx = lib().orc_argmax(score, ptr, score.size, ctypes.byref(val))
    return int(idx), float(val.value)


def find_contours_external(img):
    """cv::findContours(img, RETR_EXTERNAL, CHAIN_APPROX_NONE) restated.
    Returns a list of (k, 2) int arrays of (x, y) points, OpenCV order."""
    img = _c(img, np.uint8)
    h, w = img.shape
    pcap = 8 * w * h + 16
    ccap = w * h + 1
    pts = np.empty(2 * pcap, np.int32)
    st = np.empty(ccap + 1, np.int64)
    nc = lib().orc_find_contours_external(img, w, h, pts, pcap, st, ccap)
    if nc < 0:
        raise RuntimeError("oracle contour capacity exceeded")
    pts = pts.reshape(-1, 2)
    return [pts[st[c]:st[c + 1]].copy() for c in range(nc)]


def find_safety_contour_indices(Dx, Dy, safe, width, height):
    Dx = _c(Dx, np.float64); Dy = _c(Dy, np.float64); safe = _c(safe, np.uint8)
    cap = 8 * width * height + 16
    out = np.empty(cap, np.int32)
    n = lib().orc_find_safety_contour_indices(Dx, Dy, safe, Dx.size, int(width), int(height), out, cap)
    if n < 0:
        raise RuntimeError("oracle frontier capacity exceeded")
    return out[:n].copy()


def next_subgoal(Dx, Dy, lo, hi, safe, width, height, gx=0.0, gy=0.0):
    return int(lib().orc_next_subgoal(_c(Dx, np.float64), _c(Dy, np.float64), _c(lo, np.float64),
                                      _c(hi, np.float64), _c(safe, np.uint8), len(Dx),
                                      int(width), int(height), float(gx), float(gy)))


# ------------------------------------------ post-selection geometry (8(f)4)
# Pure-Python restatements (IEEE double, no FMA: the same roundings as the
# reference's plain C++ double arithmetic).  Small rings only.
def ring_area2(x, y):
    """Twice the signed area of a closed ring (> 0 counter-clockwise)."""
    s = 0.0
    for i in range(len(x) - 1):
        s += float(x[i]) * float(y[i + 1]) - float(x[i + 1]) * float(y[i])
    return s


def polygon_correct(x, y):
    """bg::correct for polygon<point, false, true> (node :682): close an open
    ring of > 2 points, reverse a clockwise one."""
    x = [float(v) for v in x]
    y = [float(v) for v in y]
    if len(x) > 2 and (x[0] != x[-1] or y[0] != y[-1]):
        x.append(x[0])
        y.append(y[0])
    if ring_area2(x, y) < 0.0:
        x.reverse()
        y.reverse()
    return np.array(x, np.float64), np.array(y, np.float64)


def polydist(x, y, px, py):
    """polydist, src/libraries/polygeom_lib.cpp:401-474, line by line:
    closing point dropped (:431), dxy/diff_norm with the wrap and 0 -> 1
    (:434-447), w clamped to [0, 1] and the candidate blended from
    VertexList[i] and VertexListRolled[i] == VertexList[i] (:439-440, :453-461),
    first minimum of the distances (:465-468).  None for an empty ring (the
    reference's :420-431 ends in pop_back on an empty vector)."""
    import math
    if len(x) <= 1:
        return None
    V = [(float(x[i]), float(y[i])) for i in range(len(x) - 1)]
    n = len(V)
    dxy = [(0.0, 0.0)] * n
    dn = [0.0] * n
    for i in range(n):
        j = (i + 1) % n
        dxy[j] = (V[j][0] - V[i][0], V[j][1] - V[i][1])
        d = math.sqrt(dxy[j][0] * dxy[j][0] + dxy[j][1] * dxy[j][1])
        dn[j] = 1.0 if d == 0.0 else d
    px, py = float(px), float(py)
    best = None
    for i in range(n):
        n2 = dn[i] * dn[i]
        wt = (px - V[i][0]) * (dxy[i][0] / n2) + (py - V[i][1]) * (dxy[i][1] / n2)
        w = max(min(wt, 1.0), 0.0)
        cx = (1 - w) * V[i][0] + w * V[i][0]
        cy = (1 - w) * V[i][1] + w * V[i][1]
        ex, ey = px - cx, py - cy
        d = math.sqrt(ex * ex + ey * ey)
        if best is None or d < best[2]:
            best = (cx, cy, d)
    return best


def point_within(x, y, px, py):
    """bg::within(point, polygon) (node :657): winding number, boundary -> 0."""
    n = len(x)
    if n < 3:
        return 0
    wn = 0
    for i in range(n):
        j = (i + 1) % n
        ax, ay, bx, by = float(x[i]), float(y[i]), float(x[j]), float(y[j])
        if ax == bx and ay == by:
            continue
        s = (bx - ax) * (py - ay) - (by - ay) * (px - ax)
        if s == 0.0 and min(ax, bx) <= px <= max(ax, bx) and min(ay, by) <= py <= max(ay, by):
            return 0
        if ay <= py:
            if by > py and s > 0.0:
                wn += 1
        elif by <= py and s < 0.0:
            wn -= 1
    return int(wn != 0)


# ------------------------------------------- Eigen-class CPU path (bench only)
class BlasPredictor:
    """The dense CPU predictive path a node would run on its host with Eigen
    (``LLT::matrixL().solve(K*^T)`` is a blocked TRSM, SURVEY.md 8(d) CPU
    comparator): given the lower factor L (f32) and alpha, for each block of
    queries build K*^T (N x k, f32, orc_cross_kernel_f32 on every OpenMP
    thread), mu = m0 + K*^T alpha (sgemv),
    V = L^-1 K*^T by OpenBLAS ``strsm`` (level-3, multithreaded), var = sf2 -
    colsum(V^2); then ComputeSets + argmax (orc_compute_sets / orc_argmax).
    Dense: no tile skipping.  TEST/BENCH INFRASTRUCTURE: only bench.py's
    cpu_baseline leg uses it, as the timed CPU comparator."""

    def __init__(self, L, alpha, x, y, ell, sf2, m0, block=2048):
        self.Lf = np.asfortranarray(L, dtype=np.float32)       # lower factor, Fortran order for strsm
        self.alpha = np.ascontiguousarray(alpha, np.float32)
        self.x = np.ascontiguousarray(x, np.float32)[:, None]
        self.y = np.ascontiguousarray(y, np.float32)[:, None]
        self.ell = float(ell)
        self.sf2, self.m0 = np.float32(sf2), np.float32(m0)
        self.block = int(block)

    def predict(self, qx, qy):
        from scipy.linalg.blas import strsm
        qx = np.ascontiguousarray(qx, np.float32)
        qy = np.ascontiguousarray(qy, np.float32)
        m = qx.size
        n = self.x.size
        mu = np.empty(m, np.float32)
        var = np.empty(m, np.float32)
        K = np.empty((n, self.block), np.float32, order="F")
        for a in range(0, m, self.block):
            b = min(m, a + self.block)
            Kb = K[:, : b - a]
            # K*^T of the block on every thread (orc_cross_kernel_f32, OpenMP)
            lib().orc_cross_kernel_f32(self.x.ravel(), self.y.ravel(), n, qx[a:b], qy[a:b], b - a, self.ell,
                                       self.sf2, Kb.ctypes.data)
            mu[a:b] = self.m0 + self.alpha @ Kb
            V = strsm(1.0, self.Lf, Kb, lower=1, overwrite_b=1)
            var[a:b] = np.maximum(self.sf2 - np.einsum("ij,ij->j", V, V), 0.0)
        return mu, var

    def tick(self, qx, qy, beta, f_min):
        mu, var = self.predict(qx, qy)
        lo, hi, s = compute_sets(mu, np.sqrt(var), beta, f_min)
        return argmax(hi - lo, s)
