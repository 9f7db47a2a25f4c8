"""Probe (GPU): how the query blocks' shape changes the plan on a regular
grid.  Sweeps the C4 (or --config) grid in the library's default order
(SBO_OPT_QUERY_ORDER 1: grid patches for a raster grid), in its Morton order
(2) and, with SBO_OPT_QUERY_ORDER 0, in caller-built 16 x 8 / 8 x 16 grid
patches (patches in Morton / raster order; partial patches padded with
their nearest grid point), and prints sweep time, kept tiles and levels.

  python tools/patch_order_probe.py --config C4 --rounds 3"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def spread(v):
    v = v.astype(np.uint64) & 0xFFFF
    v = (v | (v << 8)) & 0x00FF00FF
    v = (v | (v << 4)) & 0x0F0F0F0F
    v = (v | (v << 2)) & 0x33333333
    v = (v | (v << 1)) & 0x55555555
    return v


def patch_arrays(qx, qy, pw, ph, order):
    gx, gy = np.unique(qx), np.unique(qy)
    W, H = gx.size, gy.size
    assert W * H == qx.size
    npx, npy = (W + pw - 1) // pw, (H + ph - 1) // ph
    px, py = np.meshgrid(np.arange(npx), np.arange(npy))
    px, py = px.ravel(), py.ravel()
    key = spread(px) | (spread(py) << 1) if order == "morton" else py * npx + px
    o = np.argsort(key, kind="stable")
    px, py = px[o], py[o]
    lx, ly = np.meshgrid(np.arange(pw), np.arange(ph))
    ix = np.minimum(px[:, None] * pw + lx.ravel()[None, :], W - 1)
    iy = np.minimum(py[:, None] * ph + ly.ravel()[None, :], H - 1)
    return gx[ix.ravel()].astype(np.float32), gy[iy.ravel()].astype(np.float32)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="C4")
    p.add_argument("--rounds", type=int, default=3)
    a = p.parse_args()
    import torch
    from safe_bayesian_optimization_amd import TerrainMapper, synthetic
    from safe_bayesian_optimization_amd import _native as N
    from safe_bayesian_optimization_amd.terrain import CONFIGS
    n, gw, gh = CONFIGS[a.config]
    wl = synthetic(n, gw, gh, seed=0, name=a.config)
    dev = torch.device("cuda:0")
    t = lambda v: torch.as_tensor(np.ascontiguousarray(v, np.float32), device=dev)  # noqa: E731
    gm = TerrainMapper(0, wl.hyper)
    gm.fit(t(wl.x), t(wl.y), t(wl.obs))
    lib = N.lib()
    cases = [("library default (1)", 1, wl.qx, wl.qy), ("library Morton (2)", 2, wl.qx, wl.qy)]
    for pw, ph in ((16, 8), (8, 16)):
        for order in ("morton", "raster"):
            x, y = patch_arrays(wl.qx, wl.qy, pw, ph, order)
            cases.append((f"patch {pw}x{ph} {order}", 0, x, y))
    for name, qo, x, y in cases:
        gm.set_option(N.SBO_OPT_QUERY_ORDER, qo)
        qx, qy = t(x), t(y)
        m = qx.numel()
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
        ms = np.median([z[0] for z in res])
        tiles = res[-1][1] / (2 * 256 * 128 * 64)
        print(f"{name:24s} M {m:8d}  sweep {ms:6.2f} ms  ({ms * 1e6 / wl.qx.size:.2f} ns per grid point)  "
              f"tiles {tiles:.4g}  levels {res[-1][2]}", flush=True)
    gm.set_option(N.SBO_OPT_QUERY_ORDER, 1)
    gm.close()


if __name__ == "__main__":
    main()
