"""A/B of the precise sweep's two kernels (SBO_OPT_PRECISE_KERNEL 0: f64 MFMA,
1: int8 sliced) on the lpsc.yaml box at N (default 16384) and the bench's
1000 x 1000 grid: ms per tick (HIP events of the sweep launch, sbo_profile),
and the variance / mean error of each against the fp64 oracle given the
device factor on a sample.  GPU diagnostic (tools/), one JSON line.
OZ_KERNELS: the kernels (default "1 0"); TABLE_MB: SBO_OPT_TABLE_MB; INV_OZ:
SBO_OPT_INV_OZ (the fit's inverse by the int8-sliced GEMM).
    python tools/oz_ab.py [n] [sample]"""
import ctypes
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
    ns = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    O.set_threads(16)
    dev = torch.device("cuda:0")
    wl = synthetic_box(n, 1000, 1000, seed=0)
    h = wl.hyper
    gm = TerrainMapper(0, h)
    t = lambda a: torch.tensor(f32(a), device=dev)  # noqa: E731
    res = {"n": n}
    kernels = [int(k) for k in os.environ.get("OZ_KERNELS", "1 0").split()]
    if os.environ.get("TABLE_MB"):
        gm.set_option(N.SBO_OPT_TABLE_MB, int(os.environ["TABLE_MB"]))
    if os.environ.get("INV_OZ"):
        gm.set_option(N.SBO_OPT_INV_OZ, int(os.environ["INV_OZ"]))
    for kernel in kernels:
        gm.set_option(N.SBO_OPT_PRECISE_KERNEL, kernel)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gm.fit(t(wl.x), t(wl.y), t(wl.obs))
        torch.cuda.synchronize()
        fit_ms = (time.perf_counter() - t0) * 1e3
        qx, qy = t(wl.qx), t(wl.qy)
        mu, sd = gm.predict(qx, qy)            # warm
        lib = N.lib()
        lib.sbo_profile(gm.ctx.handle, 1)
        reps = 2
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            mu, sd = gm.predict(qx, qy)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / reps
        pm, pl = ctypes.c_double(), ctypes.c_int64()
        fm, fl = ctypes.c_double(), ctypes.c_int64()
        lib.sbo_profile_read(gm.ctx.handle, ctypes.byref(pm), ctypes.byref(pl), ctypes.byref(fm), ctypes.byref(fl))
        w = ctypes.c_double()
        lib.sbo_profile_work(gm.ctx.handle, ctypes.byref(w))
        lib.sbo_profile(gm.ctx.handle, 0)
        res[f"kernel{kernel}"] = {"fit_ms": fit_ms, "tick_ms": wall * 1e3, "sweep_ms": pm.value / max(pl.value, 1),
                                  "flops_per_launch": w.value / max(pl.value, 1),
                                  "precise": gm.precision()[0], "mu": mu.cpu().numpy(), "sd": sd.cpu().numpy()}
        print(f"kernel {kernel}: fit {fit_ms:.1f} ms, tick {wall * 1e3:.1f} ms, sweep {res[f'kernel{kernel}']['sweep_ms']:.1f} ms",
              flush=True)
    sel = np.sort(np.random.default_rng(3).choice(wl.qx.size, ns, replace=False))
    L, alpha = gm.factor()
    o = gm.order()
    from scipy.linalg import solve_triangular
    L64 = L.astype(np.float64)
    r = f32(wl.obs)[o].astype(np.float64) - h.prior_mean
    a64 = solve_triangular(L64.T, solve_triangular(L64, r, lower=True), lower=False)
    omu, ovar = O.predict(O.colmajor_from_lower(L64), a64, f32(wl.x)[o], f32(wl.y)[o], f32(wl.qx[sel]),
                          f32(wl.qy[sel]), h.length_scale, h.sf2, h.prior_mean)
    out = {"n": n, "sample": ns}
    for kernel in kernels:
        r_ = res[f"kernel{kernel}"]
        out[f"kernel{kernel}"] = {k: v for k, v in r_.items() if k not in ("mu", "sd")}
        out[f"kernel{kernel}"]["mu_err"] = nrel(r_["mu"][sel], omu)
        out[f"kernel{kernel}"]["var_err"] = nrel(r_["sd"][sel].astype(np.float64) ** 2, ovar)
    if "kernel0" in res and "kernel1" in res:
        v1 = res["kernel1"]["sd"].astype(np.float64) ** 2
        v0 = res["kernel0"]["sd"].astype(np.float64) ** 2
        out["int8_vs_f64_whole_grid_var"] = nrel(v1, v0)
        out["int8_vs_f64_whole_grid_mu"] = nrel(res["kernel1"]["mu"], res["kernel0"]["mu"].astype(np.float64))
        out["speedup"] = out["kernel0"]["sweep_ms"] / out["kernel1"]["sweep_ms"]
    if "kernel3" in res and "kernel4" in res:   # round 5: the k-tile pair sweep against the table sweep
        v3 = res["kernel3"]["sd"].astype(np.float64) ** 2
        v4 = res["kernel4"]["sd"].astype(np.float64) ** 2
        out["pair_vs_table_whole_grid_var"] = nrel(v4, v3)
        out["pair_vs_table_whole_grid_mu"] = nrel(res["kernel4"]["mu"], res["kernel3"]["mu"].astype(np.float64))
        out["pair_speedup"] = out["kernel3"]["sweep_ms"] / out["kernel4"]["sweep_ms"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
