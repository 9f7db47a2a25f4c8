"""Where does the predictive variance error come from?  (diagnostic, GPU)

For one workload: device result vs the fp64 oracle given the device L, and the
same sweep recomputed on the host in f64 from the device's packed operand
A = sf2 L^-1 (isolates the inverse/rounding of A from the kernel's K* and
accumulation error)."""
import ctypes
import sys
import os

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402
from safe_bayesian_optimization_amd import TerrainMapper, synthetic  # noqa: E402
from safe_bayesian_optimization_amd import _native as N  # noqa: E402
from safe_bayesian_optimization_amd.terrain import Hyper  # noqa: E402


def nrel(a, b):
    return float(np.abs(np.asarray(a, np.float64) - b).max() / np.abs(b).max())


def diag(wl, nq=2048):
    h = wl.hyper
    sel = np.random.default_rng(0).choice(wl.qx.size, min(nq, wl.qx.size), replace=False)
    qx, qy = wl.qx[sel].astype(np.float32), wl.qy[sel].astype(np.float32)
    x, y = wl.x.astype(np.float32), wl.y.astype(np.float32)
    for bits in (32, 64):
        gm = TerrainMapper(0, h)
        gm.ctx.check(N.lib().sbo_set_option(gm.ctx.handle, N.SBO_OPT_INVERSE_BITS, bits))
        gm.fit(x, y, wl.obs.astype(np.float32))
        mu, sd = gm.predict(qx, qy)
        L, alpha = gm.factor()
        o = gm.order()  # factor rows are in the library's internal (Morton) order
        n = L.shape[0]
        xo, yo = x[o], y[o]
        omu, ovar = O.predict(O.colmajor_from_lower(L.astype(np.float64)), alpha.astype(np.float64), xo, yo, qx, qy,
                              h.length_scale, h.sf2, h.prior_mean)
        A = np.zeros((n, n), np.float32)
        gm.ctx.check(N.lib().sbo_get_inverse(gm.ctx.handle, A.ctypes.data))
        A = np.tril(A).astype(np.float64)
        inv_err = np.abs(A @ L.astype(np.float64) / h.sf2 - np.eye(n)).max()
        xs, ys = xo.astype(np.float64), yo.astype(np.float64)
        E = np.exp(-((xs[:, None] - qx[None, :].astype(np.float64)) ** 2 + (ys[:, None] - qy[None, :].astype(np.float64)) ** 2)
                   / (2 * h.length_scale ** 2))
        V = A @ E
        hvar = h.sf2 - (V * V).sum(0)
        print(f"N={n} bits={bits}: device mu {nrel(mu, omu):.2e} var {nrel(sd.astype(np.float64)**2, ovar):.2e} | "
              f"host f64 sweep from device A: var {nrel(hvar, ovar):.2e} | max|A L/sf2 - I| {inv_err:.2e}", flush=True)
        gm.close()


if __name__ == "__main__":
    diag(synthetic(700, 50, 20, seed=3, hyper=Hyper(0.7, 1.7, 0.05, 0.3)))
    diag(synthetic(2048, 64, 64, seed=2055))
    diag(synthetic(8192, 1024, 1024, seed=0))
