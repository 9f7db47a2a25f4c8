"""Accuracy of the posterior on the mapping node's own box (config/lpsc.yaml:32-37):
N points on x [0, 1] x y [0, 2.5], l = 0.4, sigma_f = 1, noise 0.1, on the
bench's 1000 x 1000 grid and the mapper's resolution [300, 120] grid.

For a 3072-point sample: mu / sigma^2 normwise error against the fp64 oracle
given the device factor, for the default sweep and diagnostic variants, with
the f32 strtrs / sgemv yardsticks (the reference implementation class) and
the error a host f64 sweep of the device's own f32 operand A = sf2 L^-1 has.
GPU diagnostic (tools/), prints one JSON line per case."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from oracle import oracle as O  # noqa: E402
from safe_bayesian_optimization_amd import TerrainMapper  # noqa: E402
from safe_bayesian_optimization_amd import _native as N  # noqa: E402
from safe_bayesian_optimization_amd.terrain import synthetic_box  # noqa: E402


def f32(a):
    return np.ascontiguousarray(a, np.float32)


def nrel(a, b):
    return float(np.abs(np.asarray(a, np.float64) - b).max() / max(np.abs(b).max(), 1e-30))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    grids = [(1000, 1000), (300, 120)]
    dev = torch.device("cuda:0")
    O.set_threads(16)
    for gw, gh in grids:
        wl = synthetic_box(n, gw, gh, seed=0)
        h = wl.hyper
        gm = TerrainMapper(0, h)
        t = lambda a: torch.tensor(f32(a), device=dev)  # noqa: E731
        t0 = time.perf_counter()
        gm.fit(t(wl.x), t(wl.y), t(wl.obs))
        torch.cuda.synchronize()
        fit_s = time.perf_counter() - t0
        m = wl.qx.size
        sel = np.sort(np.random.default_rng(7).choice(m, min(3072, m), replace=False))
        L, alpha = gm.factor()
        o = gm.order()
        xs, ys = f32(wl.x)[o], f32(wl.y)[o]
        Lcm = O.colmajor_from_lower(L.astype(np.float64))
        omu, ovar = O.predict(Lcm, alpha.astype(np.float64), xs, ys, f32(wl.qx[sel]), f32(wl.qy[sel]),
                              h.length_scale, h.sf2, h.prior_mean)
        del Lcm
        # yardsticks: f32 strtrs on the same L, the same f32 K*; f32 sgemv mean
        import scipy.linalg as sla
        qx64, qy64 = f32(wl.qx[sel]).astype(np.float64), f32(wl.qy[sel]).astype(np.float64)
        E = np.exp(-((xs.astype(np.float64)[:, None] - qx64[None, :]) ** 2
                     + (ys.astype(np.float64)[:, None] - qy64[None, :]) ** 2) / (2 * h.length_scale ** 2))
        Ks = (h.sf2 * E).astype(np.float32)
        V = sla.solve_triangular(L, Ks, lower=True).astype(np.float64)
        e_strtrs = nrel(h.sf2 - (V * V).sum(0), ovar)
        del V
        mu32 = np.float32(h.prior_mean) + E.astype(np.float32).T @ (np.float32(h.sf2) * alpha.astype(np.float32))
        e_sgemv = nrel(mu32.astype(np.float64), omu)
        # host f64 sweep of the device's own f32 operand A = sf2 L^-1 (exact K*)
        A = np.empty((n, n), np.float32)
        gm.ctx.check(N.lib().sbo_get_inverse(gm.ctx.handle, A.ctypes.data_as(__import__("ctypes").c_void_p)))
        A64 = np.tril(A).astype(np.float64)
        del A
        Vd = A64 @ E
        e_opnd = nrel(h.sf2 - (Vd * Vd).sum(0), ovar)
        del A64, Vd, E, Ks
        res = {"n": n, "grid": [gw, gh], "fit_s": fit_s, "cutoff": gm.skip_info()[0],
               "var_max": float(ovar.max()), "var_min": float(ovar.min()), "var_median": float(np.median(ovar)),
               "mu_absmax": float(np.abs(omu).max()), "alpha_l1": float(np.abs(alpha).sum()),
               "strtrs_var": e_strtrs, "sgemv_mu": e_sgemv, "f64_sweep_of_f32_operand_var": e_opnd}
        qx, qy = t(wl.qx), t(wl.qy)
        for name, opts in (("default", {}), ("v22_dense", {N.SBO_OPT_KERNEL_VARIANT: 22, N.SBO_OPT_TILE_SKIP: 0}),
                           ("v0_f32_dense", {N.SBO_OPT_KERNEL_VARIANT: 0, N.SBO_OPT_TILE_SKIP: 0})):
            for k, v in opts.items():
                gm.set_option(k, v)
            mu, sd = gm.predict(qx, qy)
            torch.cuda.synchronize()
            mu, sd = mu.cpu().numpy(), sd.cpu().numpy()
            res[name] = {"mu": nrel(mu[sel], omu), "var": nrel(sd[sel].astype(np.float64) ** 2, ovar),
                         "var_abs": float(np.abs(sd[sel].astype(np.float64) ** 2 - ovar).max())}
            gm.set_option(N.SBO_OPT_KERNEL_VARIANT, 3)
            gm.set_option(N.SBO_OPT_TILE_SKIP, -1)
        print(json.dumps(res), flush=True)
        gm.close()


if __name__ == "__main__":
    main()
