"""Accuracy of predictive-kernel variants against a host f64 sweep (diagnostic, GPU).

For one workload the device operand A = sf2 L^-1 is read back and the
variance sf2 - |A k*|^2 recomputed on the host in f64 for a query sample;
each kernel variant's variance is compared with it (normwise relative, the
staged contract's measure).  This isolates the kernel's K* and accumulation
error from the factorisation error.

  python tools/variant_accuracy.py --n 8192 16384 --variants 0 1 5 6 7
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from safe_bayesian_optimization_amd import TerrainMapper, synthetic  # noqa: E402
from safe_bayesian_optimization_amd import _native as N  # noqa: E402


def nrel(a, b):
    return float(np.abs(np.asarray(a, np.float64) - b).max() / np.abs(b).max())


def run(n, variants, nq, skip, budget=None):
    wl = synthetic(n, 1000, 1000, seed=0)
    h = wl.hyper
    rng = np.random.default_rng(1)
    # a compact patch of the grid (what one Morton-ordered sweep block sees) plus scattered points
    sel = np.concatenate([np.arange(nq // 2) + wl.qx.size // 3, rng.choice(wl.qx.size, nq - nq // 2, replace=False)])
    qx, qy = wl.qx[sel].astype(np.float32), wl.qy[sel].astype(np.float32)
    gm = TerrainMapper(0, h)
    gm.set_option(N.SBO_OPT_TILE_SKIP, skip)
    if budget is not None:
        gm.set_option(N.SBO_OPT_SKIP_BUDGET, budget)
    gm.fit(wl.x.astype(np.float32), wl.y.astype(np.float32), wl.obs.astype(np.float32))
    A = np.zeros((n, n), np.float32)
    gm.ctx.check(N.lib().sbo_get_inverse(gm.ctx.handle, A.ctypes.data))
    A = np.tril(A).astype(np.float64)
    o = gm.order()
    xs, ys = wl.x[o].astype(np.float32).astype(np.float64), wl.y[o].astype(np.float32).astype(np.float64)
    E = np.exp(-((xs[:, None] - qx[None, :].astype(np.float64)) ** 2 +
                 (ys[:, None] - qy[None, :].astype(np.float64)) ** 2) / (2 * h.length_scale ** 2))
    V = A @ E
    hvar = h.sf2 - (V * V).sum(0)
    Lf, alpha = gm.factor()
    hmu = h.prior_mean + h.sf2 * (E.T @ alpha.astype(np.float64))
    del A, E, V
    for v in variants:
        gm.set_option(N.SBO_OPT_KERNEL_VARIANT, v)
        mu, sd = gm.predict(qx, qy)
        var = sd.astype(np.float64) ** 2
        L = gm.skip_info()[0]
        print(f"N={n} skip={skip} budget={budget} (L={L}) variant {v}: var vs host f64 sweep {nrel(var, hvar):.2e}"
              f"  mu vs host f64 {nrel(mu, hmu):.2e}", flush=True)
    gm.close()


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, nargs="+", default=[8192, 16384])
    p.add_argument("--variants", type=int, nargs="+", default=[0, 1])
    p.add_argument("--nq", type=int, default=1024)
    p.add_argument("--skip", type=int, default=-1)
    p.add_argument("--budget", type=int, nargs="*", default=[None])
    a = p.parse_args()
    for n in a.n:
        for b in a.budget:
            run(n, a.variants, a.nq, a.skip, b)


if __name__ == "__main__":
    main()
