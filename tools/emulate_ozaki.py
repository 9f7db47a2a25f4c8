"""Host emulation of an Ozaki-style sliced product for the precise sweep
(VERDICT r3 next-2): V = A K*, A = sf2 L^-1 (f64, the fit's inverse), K* in
f64, both cut into int8 digit slices with a power-of-two scale per block, the
slice products accumulated exactly (int32 on the device: here f64 matmuls of
integer-valued operands, exact below 2^53) and combined in f64 per k-tile.

Measures the normwise variance error against the f64 solve on the lpsc.yaml box
(the regime where the fast sweep misses the 1e-5 contract by 40x) for
  - P digits per operand, products kept where s + u < P (triangular) or all;
  - the A scale per (row, k-tile), per (16-row block, k-tile) or per (256-row
    block, k-tile); the K* scale per (query, k-tile);
  - digits by truncation or by rounding (|digit| <= 127 either way).
Mode "kernel" (third argument) emulates predict_oz_kernel's final scheme
instead: balanced base-256 digits from integers (XA = rint(A 2^(39 - eA)),
five digits; X = rint(K* 2^(31 - eK)), four digits; 2^e > 1.01 max per block),
the 14 pairs s + u <= 4 (u <= 3), level 4 rounded to level-3 units, next to
the round-4 base-128 form (five A digits, four K* digits, s + u <= 4).
CPU only (numpy/scipy, ~12 GB at n = 16384, a few minutes):
    python tools/emulate_ozaki.py [n] [queries] [kernel]"""
import os
import sys
import time

import numpy as np
import scipy.linalg as sla

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402
from safe_bayesian_optimization_amd.terrain import synthetic_box  # noqa: E402

BK = 64


def digits(x, P, mode):
    """x in (-1, 1) (already scaled) as P base-128 digits d_s (|d_s| <= 127):
    x = sum_s d_s 128^-(s+1) + r, |r| <= 128^-P (trunc) / 128^-P / 2 (round)."""
    r = x
    out = []
    for s in range(P):
        r = r * 128.0
        d = np.trunc(r) if (mode == "trunc" or s == 0) else np.clip(np.rint(r), -127, 127)
        out.append(d)
        r = r - d
    return out


def digits256(X, P):
    """Integer X (|X| < 2^(8P - 1) / 1.01) as P balanced base-256 digits, top
    first: the bytes of X + 0x80..80 (P - 1 lower bytes), less 128 but for the top."""
    Y = X.astype(np.int64) + sum(128 << (8 * i) for i in range(P - 1))
    out = []
    for s in range(P):
        sh = 8 * (P - 1 - s)
        b = (Y >> sh) if s == 0 else ((Y >> sh) & 0xFF) - 128
        out.append(b.astype(np.float64))
    return out


def exp101(m):
    """e with 2^e > 1.01 m (frexp's exponent; 0 for m == 0)."""
    return np.where(m > 0, np.frexp(m * 1.01)[1], 0).astype(np.int64)


def scheme256(A, E, n, nq, PA, PK, Lmax):
    """Base-256 variants: PA / PK digits, pairs s + u <= Lmax (level Lmax
    rounded to units of level Lmax - 1)."""
    nt = n // BK
    eK = exp101(np.abs(E).reshape(nt, BK, nq).max(1))
    eA = np.repeat(exp101(np.abs(A).reshape(n // 16, 16, nt, BK).max(axis=(1, 3))), 16, axis=0)
    V = np.zeros((n, nq))
    npairs = sum(1 for s_ in range(PA) for u in range(PK) if s_ + u <= Lmax)
    for t in range(nt):
        ks = slice(t * BK, (t + 1) * BK)
        XA = np.rint(np.ldexp(A[:, ks], (8 * PA - 1 - eA[:, t])[:, None]))
        XK = np.rint(np.ldexp(E[ks], (8 * PK - 1 - eK[t])[None, :]))
        dA, dK = digits256(XA, PA), digits256(XK, PK)
        lv = [np.zeros((n, nq)) for _ in range(Lmax + 1)]
        for s_ in range(PA):
            for u in range(PK):
                if s_ + u <= Lmax:
                    lv[s_ + u] += dA[s_] @ dK[u]
        # sum_L lv[L] 2^(8 (PA + PK - 2 - L)), level Lmax rounded to level Lmax - 1's unit
        T = sum(lv[L] * 2.0 ** (8 * (Lmax - 1 - L)) for L in range(Lmax)) + np.rint(lv[Lmax] / 256.0)
        S = (8 * PA - 1) + (8 * PK - 1) - 8 * (PA + PK - 2 - (Lmax - 1))
        V += T * np.ldexp(1.0, (eA[:, t][:, None] + eK[t][None, :] - S))
    return V, npairs


def kernel_scheme(A, E, n, nq, base):
    """predict_oz_kernel's arithmetic: per (16-row block, k-tile) eA, per
    (k-tile, query) eK; base 256 (final) or 128 (round 4's first form)."""
    nt = n // BK
    eK = exp101(np.abs(E).reshape(nt, BK, nq).max(1))                          # (nt, nq)
    eA = np.repeat(exp101(np.abs(A).reshape(n // 16, 16, nt, BK).max(axis=(1, 3))), 16, axis=0)   # (n, nt)
    V = np.zeros((n, nq))
    for t in range(nt):
        ks = slice(t * BK, (t + 1) * BK)
        if base == 256:
            XA = np.rint(np.ldexp(A[:, ks], (39 - eA[:, t])[:, None]))
            XK = np.rint(np.ldexp(E[ks], (31 - eK[t])[None, :]))
            dA, dK, w = digits256(XA, 5), digits256(XK, 4), 8
        else:
            dA = digits(np.ldexp(A[:, ks], -eA[:, t][:, None]), 5, "round")
            dK = digits(np.ldexp(E[ks], -eK[t][None, :]), 4, "round")
            w = 7
        lv = [np.zeros((n, nq)) for _ in range(5)]
        for s_ in range(5):
            for u in range(4):
                if s_ + u <= 4:
                    lv[s_ + u] += dA[s_] @ dK[u]          # exact: integer-valued, < 2^53
        T = sum(lv[L] * 2.0 ** (w * (3 - L)) for L in range(4)) + np.rint(lv[4] / 2.0 ** w)
        # V += T 2^(eA + eK - S): base 256: S = 38 (digits weights 2^32.., 2^24..);
        # base 128: S = 35 + 0 (digits d_s 128^-(s+1): T in units of 128^-5)
        S = 38 if base == 256 else 35
        V += T * np.ldexp(1.0, (eA[:, t][:, None] + eK[t][None, :] - S))
    return V


def exp_of(m):
    """e with m < 2^e (m >= 0; 0 for m == 0)."""
    with np.errstate(divide="ignore"):
        return np.where(m > 0, np.floor(np.log2(np.where(m > 0, m, 1.0))) + 1.0, 0.0)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    nq = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    O.set_threads(8)
    wl = synthetic_box(n, 1000, 1000, seed=0)
    h = wl.hyper
    x = wl.x.astype(np.float32).astype(np.float64)
    y = wl.y.astype(np.float32).astype(np.float64)
    order = np.lexsort((y, np.floor(x * 16)))   # a spatial order (tiles compact enough for the scales)
    x, y = x[order], y[order]
    t0 = time.time()
    K = O.rbf_fill(x, y, h.length_scale, h.sf2, h.sn2).reshape(n, n)
    L = np.linalg.cholesky(K)
    del K
    A = sla.solve_triangular(L, np.eye(n), lower=True) * h.sf2
    print(f"fit {time.time() - t0:.1f} s", flush=True)
    rng = np.random.default_rng(7)
    sel = rng.choice(wl.qx.size, nq, replace=False)
    qx = wl.qx[sel].astype(np.float32).astype(np.float64)
    qy = wl.qy[sel].astype(np.float32).astype(np.float64)
    E = np.exp(-((x[:, None] - qx[None]) ** 2 + (y[:, None] - qy[None]) ** 2) / (2 * h.length_scale ** 2))
    Vt = A @ E
    var_t = h.sf2 - (Vt * Vt).sum(0)
    vmax = np.abs(var_t).max()
    print(f"var range {var_t.min():.3e} .. {vmax:.3e}", flush=True)

    def rep(name, V):
        var = h.sf2 - (V * V).sum(0)
        print(f"{name:52s} nrel {np.abs(var - var_t).max() / vmax:.3e}", flush=True)

    rep("f64 (reference, self)", Vt)
    if len(sys.argv) > 3 and sys.argv[3] == "kernel":
        rep("kernel scheme, base 128 (5 x 4 digits, 14 products)", kernel_scheme(A, E, n, nq, 128))
        rep("kernel scheme, base 256 (5 x 4 digits, 14 products)", kernel_scheme(A, E, n, nq, 256))
        for PA, PK, Lm in ((5, 4, 4), (4, 4, 4), (4, 4, 3), (5, 4, 3), (4, 3, 3), (3, 4, 3), (4, 3, 2)):
            V, npairs = scheme256(A, E, n, nq, PA, PK, Lm)
            rep(f"base 256, A {PA} x K* {PK} digits, s + u <= {Lm} ({npairs} products)", V)
        return
    A32 = A.astype(np.float32).astype(np.float64)
    rep("A rounded to f32, exact arithmetic", A32 @ E)
    E32 = E.astype(np.float32).astype(np.float64)
    rep("K* rounded to f32, exact arithmetic", A @ E32)
    nt = n // BK
    eK = exp_of(np.abs(E).reshape(nt, BK, nq).max(1))            # (nt, nq): per (k-tile, query)
    for a_grp in (1, 16, 256):
        eA = exp_of(np.abs(A).reshape(n // a_grp, a_grp, nt, BK).max(axis=(1, 3)))   # (n / grp, nt)
        eA = np.repeat(eA, a_grp, axis=0)                                          # (n, nt)
        for mode in ("trunc", "round"):
            for P in (3, 4, 5):
                V = np.zeros_like(Vt)
                Vfull = np.zeros_like(Vt)
                for t in range(nt):
                    ks = slice(t * BK, (t + 1) * BK)
                    sA = np.ldexp(1.0, eA[:, t].astype(np.int64))
                    sK = np.ldexp(1.0, eK[t].astype(np.int64))
                    dA = digits(A[:, ks] / sA[:, None], P, mode)
                    dK = digits(E[ks] / sK[None, :], P, mode)
                    acc = np.zeros((n, nq))
                    accf = np.zeros((n, nq))
                    kf = sum(dK[u] * 128.0 ** -(u + 1) for u in range(P))
                    for s in range(P):
                        kt = sum(dK[u] * 128.0 ** -(u + 1) for u in range(P - s))
                        acc += (dA[s] @ kt) * 128.0 ** -(s + 1)
                        accf += (dA[s] @ kf) * 128.0 ** -(s + 1)
                    V += acc * sA[:, None] * sK[None, :]
                    Vfull += accf * sA[:, None] * sK[None, :]
                rep(f"A grp {a_grp:3d} rows, {mode:5s}, P={P} triangular ({P * (P + 1) // 2} products)", V)
                rep(f"A grp {a_grp:3d} rows, {mode:5s}, P={P} all pairs ({P * P} products)", Vfull)


if __name__ == "__main__":
    main()
