"""Probe (GPU): the training order's effect on the plan and the sweep --
Hilbert (SBO_OPT_SPATIAL_ORDER 1), Morton (2), k-d bisection (3): fit time,
sweep time, kept tiles and levels, and mu / sigma^2 against order 1.

  python tools/spatial_order_probe.py --config C4 --rounds 3"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="C4")
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--orders", type=int, nargs="+", default=[1, 3, 2])
    a = p.parse_args()
    import torch
    from safe_bayesian_optimization_amd import TerrainMapper, synthetic
    from safe_bayesian_optimization_amd import _native as N
    from safe_bayesian_optimization_amd.terrain import CONFIGS
    n, gw, gh = CONFIGS[a.config]
    wl = synthetic(n, gw, gh, seed=0, name=a.config)
    dev = torch.device("cuda:0")
    t = lambda v: torch.as_tensor(np.ascontiguousarray(v, np.float32), device=dev)  # noqa: E731
    qx, qy = t(wl.qx), t(wl.qy)
    m = qx.numel()
    lib = N.lib()
    ref = None
    for order in a.orders:
        gm = TerrainMapper(0, wl.hyper)
        gm.set_option(N.SBO_OPT_SPATIAL_ORDER, order)
        gm.fit(t(wl.x), t(wl.y), t(wl.obs))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gm.fit(t(wl.x), t(wl.y), t(wl.obs))
        torch.cuda.synchronize()
        fit_ms = (time.perf_counter() - t0) * 1e3
        res = []
        for r in range(a.rounds + 1):
            mu = torch.empty(m, device=dev)
            sd = torch.empty(m, device=dev)
            lib.sbo_profile(gm.ctx.handle, 1)
            gm.tick(qx, qy, wl.beta, wl.f_min, outputs=dict(mu=mu, sd=sd))
            pm, pl, fm, fl = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_int64()
            lib.sbo_profile_read(gm.ctx.handle, ctypes.byref(pm), ctypes.byref(pl), ctypes.byref(fm), ctypes.byref(fl))
            w, mf = ctypes.c_double(), ctypes.c_double()
            lib.sbo_profile_work(gm.ctx.handle, ctypes.byref(w))
            lv = (ctypes.c_int64 * 3)()
            lib.sbo_profile_mfma(gm.ctx.handle, ctypes.byref(mf), lv)
            if r:
                res.append((pm.value, w.value, list(lv)))
        out = (mu.cpu().numpy().astype(np.float64), sd.cpu().numpy().astype(np.float64) ** 2)
        if ref is None:
            ref = out
        emu = np.abs(out[0] - ref[0]).max() / np.abs(ref[0]).max()
        evar = np.abs(out[1] - ref[1]).max() / np.abs(ref[1]).max()
        ms = np.median([z[0] for z in res])
        print(f"order {order}: fit {fit_ms:6.1f} ms  sweep {ms:6.2f} ms  tiles {res[-1][1] / (2 * 256 * 128 * 64):.4g}  "
              f"levels {res[-1][2]}  | mu {emu:.2e} var {evar:.2e} vs order {a.orders[0]}", flush=True)
        gm.close()


if __name__ == "__main__":
    main()
