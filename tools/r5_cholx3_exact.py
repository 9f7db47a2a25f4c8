"""Round 5: is the split-bf16 Cholesky's factor (SBO_OPT_CHOL_GEMM 3) as good
as rocBLAS's (0)?  Both fits' posteriors (default options: whichever sweep
the probe picks) against the exact one -- the fp64 oracle over an f64
Cholesky of K in f64 (numpy), alpha in f64 -- on a sample of the grid, with
each factor's backward error ||L L^T - K|| / ||K||.  GPU diagnostic:
CHOL_GEMMS / OUTERS: the SBO_OPT_CHOL_GEMM / SBO_OPT_CHOL_OUTER values.
    python tools/r5_cholx3_exact.py [n] [sample]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from oracle import oracle as O  # noqa: E402
from safe_bayesian_optimization_amd import TerrainMapper, synthetic  # noqa: E402
from safe_bayesian_optimization_amd import _native as N  # noqa: E402
from safe_bayesian_optimization_amd.terrain import synthetic_box  # noqa: E402


def f32(a):
    return np.ascontiguousarray(a, np.float32)


def nrel(a, b):
    return float(np.abs(np.asarray(a, np.float64) - b).max() / max(np.abs(b).max(), 1e-30))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    ns = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    O.set_threads(16)
    rng = np.random.default_rng(5)
    for name, wl in (("C3-like", synthetic(n, 500, 500, seed=1)), ("lpsc box", synthetic_box(n, 500, 500, seed=1))):
        h = wl.hyper
        sel = np.sort(rng.choice(wl.qx.size, ns, replace=False))
        qx, qy = f32(wl.qx[sel]), f32(wl.qy[sel])
        exact = None
        for g, ou in [(int(v), int(u)) for v in os.environ.get("CHOL_GEMMS", "0 3").split()
                      for u in os.environ.get("OUTERS", "512").split()]:
            gm = TerrainMapper(0, h)
            gm.set_option(N.SBO_OPT_CHOL_GEMM, g)
            gm.set_option(N.SBO_OPT_CHOL_OUTER, ou)
            gm.fit(wl.x, wl.y, wl.obs)
            o = gm.order()
            L, _ = gm.factor()
            mu, sd = gm.predict(wl.qx, wl.qy)
            precise = gm.precision()[0]
            gm.close()
            K = O.rbf_fill_f32in(f32(wl.x)[o], f32(wl.y)[o])
            L64 = L.astype(np.float64)
            be = np.linalg.norm(L64 @ L64.T - K) / np.linalg.norm(K)
            if exact is None:
                Le = np.linalg.cholesky(K)
                r = f32(wl.obs)[o].astype(np.float64) - h.prior_mean
                from scipy.linalg import solve_triangular
                alpha = solve_triangular(Le.T, solve_triangular(Le, r, lower=True), lower=False)
                exact = O.predict(O.colmajor_from_lower(Le), alpha, f32(wl.x)[o], f32(wl.y)[o], qx, qy,
                                  h.length_scale, h.sf2, h.prior_mean)
                del Le
            emu = nrel(mu[sel], exact[0])
            evar = nrel(sd[sel].astype(np.float64) ** 2, exact[1])
            print(f"{name} N={n} chol_gemm={g} outer={ou}: backward error {be:.2e}; vs the exact posterior: mu {emu:.2e} "
                  f"var {evar:.2e} (precise sweep {precise})", flush=True)


if __name__ == "__main__":
    main()
