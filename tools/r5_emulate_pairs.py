"""Host emulation (round 5): the int8 sliced precise sweep
with its exponents shared over a GROUP of G consecutive k-tiles, so that the
int32 level sums chain over 64 G k before one f64 combination (the
combination's VALU is what bounds predict_oz_kernel: profiles/r5_pmc_oz_table.txt,
25.8 % VALU instructions against 6.2 % MFMA, matrix pipe 48 %).

predict_oz_kernel's arithmetic (tools/r4_emulate_ozaki.py, "kernel" mode):
  eA per (16-row block, group), eK per (query, group): 2^e > 1.01 max |.|
  XA = rint(A 2^(39 - eA)) in five balanced base-256 digits, XK = rint(K*
  2^(31 - eK)) in four, the 14 pairs s + u <= 4 summed exactly over the group's
  k, level 4 rounded to level-3 units, V += T 2^(eA + eK - 38).
Reports the normwise variance error against the f64 product (the contract is
1e-5) for G = 1 (today's kernel), 2, 4, and the int32 headroom of the
combination h23 = l2 256 + l3 + [l4 / 256] (|h23| < 2^31 needed).
CPU only:  python tools/r5_emulate_pairs.py [n] [queries]"""
import os
import sys
import time

import numpy as np
import scipy.linalg as sla

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402
from safe_bayesian_optimization_amd.terrain import synthetic_box  # noqa: E402

BK = 64


def digits256(X, P):
    Y = X.astype(np.int64) + sum(128 << (8 * i) for i in range(P - 1))
    out = []
    for s in range(P):
        sh = 8 * (P - 1 - s)
        b = (Y >> sh) if s == 0 else ((Y >> sh) & 0xFF) - 128
        out.append(b.astype(np.float64))
    return out


def exp101(m):
    return np.where(m > 0, np.frexp(m * 1.01)[1], 0).astype(np.int64)


def grouped(A, E, n, nq, G):
    nt = n // BK
    ng = nt // G
    kg = BK * G
    eK = exp101(np.abs(E).reshape(ng, kg, nq).max(1))                                       # (ng, nq)
    eA = np.repeat(exp101(np.abs(A).reshape(n // 16, 16, ng, kg).max(axis=(1, 3))), 16, axis=0)   # (n, ng)
    V = np.zeros((n, nq))
    h23max = 0.0
    for t in range(ng):
        ks = slice(t * kg, (t + 1) * kg)
        XA = np.rint(np.ldexp(A[:, ks], (39 - eA[:, t])[:, None]))
        XK = np.rint(np.ldexp(E[ks], (31 - eK[t])[None, :]))
        dA, dK = digits256(XA, 5), digits256(XK, 4)
        lv = [np.zeros((n, nq)) for _ in range(5)]
        for s_ in range(5):
            for u in range(4):
                if s_ + u <= 4:
                    lv[s_ + u] += dA[s_] @ dK[u]
        h23 = lv[2] * 256 + lv[3] + np.floor((lv[4] + 128) / 256)
        h23max = max(h23max, float(np.abs(h23).max()))
        T = (lv[0] * 256 + lv[1]) * 65536.0 + h23
        V += T * np.ldexp(1.0, (eA[:, t][:, None] + eK[t][None, :] - 38))
    return V, h23max


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    nq = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    O.set_threads(8)
    for name, sn2, ell in (("lpsc box", 0.1, 0.4), ("lpsc box sn2 0.01", 0.01, 0.4), ("lpsc box l 0.8", 0.1, 0.8)):
        wl = synthetic_box(n, 1000, 1000, seed=0)
        x = wl.x.astype(np.float32).astype(np.float64)
        y = wl.y.astype(np.float32).astype(np.float64)
        # the library's k-d order: a recursive median cut (here: a 2-level
        # column-then-row sort, compact enough for the per-tile scales)
        order = np.lexsort((y, np.floor(x * 16)))
        x, y = x[order], y[order]
        t0 = time.time()
        K = O.rbf_fill(x, y, ell, 1.0, sn2).reshape(n, n)
        L = np.linalg.cholesky(K)
        del K
        A = sla.solve_triangular(L, np.eye(n), lower=True)
        del L
        rng = np.random.default_rng(7)
        sel = rng.choice(wl.qx.size, nq, replace=False)
        qx = wl.qx[sel].astype(np.float32).astype(np.float64)
        qy = wl.qy[sel].astype(np.float32).astype(np.float64)
        E = np.exp(-((x[:, None] - qx[None]) ** 2 + (y[:, None] - qy[None]) ** 2) / (2 * ell ** 2))
        Vt = A @ E
        var_t = 1.0 - (Vt * Vt).sum(0)
        vmax = np.abs(var_t).max()
        print(f"{name}: n {n}, {nq} queries, var {var_t.min():.3e} .. {vmax:.3e} (fit {time.time() - t0:.1f} s)",
              flush=True)
        for G in (1, 2, 4):
            V, h23 = grouped(A, E, n, nq, G)
            var = 1.0 - (V * V).sum(0)
            print(f"  G = {G} tiles per exponent: var nrel {np.abs(var - var_t).max() / vmax:.3e}   "
                  f"max |h23| 2^{np.log2(max(h23, 1)):.2f}", flush=True)
        del A, E, Vt


if __name__ == "__main__":
    main()
