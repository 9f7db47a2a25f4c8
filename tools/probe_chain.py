"""Is the fit's precision probe bound by its longest work item?  Fits C4 and
sweeps the probe's query sets (a G x G lattice over the training box + MT
strided training locations) with the fast sweep (tick) and the precise one
(SBO_OPT_PRECISION 1), profiled: sweep ms and the kept tiles by level, for
several G and MT.   PK="3 0 1" python tools/probe_chain.py [n]  (PK: precise kernels)"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from safe_bayesian_optimization_amd import TerrainMapper, synthetic
    from safe_bayesian_optimization_amd import _native as N
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    dev = torch.device("cuda:0")
    wl = synthetic(n, 64, 64, seed=0)
    t = lambda v: torch.as_tensor(np.ascontiguousarray(v, np.float32), device=dev)  # noqa: E731
    X, Y, O = t(wl.x), t(wl.y), t(wl.obs)
    gm = TerrainMapper(0, wl.hyper)
    gm.fit(X, Y, O)
    lib, h = gm._lib, gm.ctx.handle
    x0, x1, y0, y1 = float(wl.x.min()), float(wl.x.max()), float(wl.y.min()), float(wl.y.max())
    kernels = [int(v) for v in os.environ.get("PK", "3").split()]
    for prec, pk in [(0, kernels[0])] + [(1, k) for k in kernels]:
        gm.set_option(N.SBO_OPT_PRECISION, prec)
        gm.set_option(N.SBO_OPT_PRECISE_KERNEL, pk)
        for G, MT in ((32, 512), (16, 512), (32, 0), (8, 128), (4, 0)):
            gx, gy = np.meshgrid(np.linspace(x0, x1, G), np.linspace(y0, y1, G))
            stride = max(n // MT, 1) if MT else 0
            tx = wl.x[stride // 2::stride][:MT] if MT else np.zeros(0)
            ty = wl.y[stride // 2::stride][:MT] if MT else np.zeros(0)
            qx, qy = t(np.concatenate([gx.ravel(), tx])), t(np.concatenate([gy.ravel(), ty]))
            ms = []
            for rep in range(3):
                lib.sbo_profile(h, 1)
                gm.tick(qx, qy, 2.0, -1.0)
                torch.cuda.synchronize()
                pm, pl, fm, fl = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_int64()
                lib.sbo_profile_read(h, ctypes.byref(pm), ctypes.byref(pl), ctypes.byref(fm), ctypes.byref(fl))
                mf = ctypes.c_double()
                lv = (ctypes.c_int64 * 3)()
                lib.sbo_profile_mfma(h, ctypes.byref(mf), lv)
                ms.append(pm.value / max(pl.value, 1))
                lib.sbo_profile(h, 0)
            print(f"N={n} {f'precise kernel {pk}' if prec else 'fast'} lattice {G}x{G} + {MT} train = {G * G + len(tx)} queries: "
                  f"sweep {min(ms):.3f} ms (of {', '.join(f'{v:.3f}' for v in ms)}), tiles by level {list(lv)}",
                  flush=True)


if __name__ == "__main__":
    main()
