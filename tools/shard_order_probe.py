"""Probe (GPU): per shard of the C4 grid (equal and plan-cost balanced cuts),
the sweep with grid patches (SBO_OPT_QUERY_ORDER 1) vs Morton (2)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from safe_bayesian_optimization_amd import TerrainMapper, synthetic
    from safe_bayesian_optimization_amd import _native as N
    from safe_bayesian_optimization_amd.dist import balanced_cuts, shard_range
    from safe_bayesian_optimization_amd.terrain import CONFIGS
    n, gw, gh = CONFIGS["C4"]
    wl = synthetic(n, gw, gh, seed=0, name="C4")
    dev = torch.device("cuda:0")
    t = lambda v: torch.as_tensor(np.ascontiguousarray(v, np.float32), device=dev)  # noqa: E731
    gm = TerrainMapper(0, wl.hyper)
    gm.fit(t(wl.x), t(wl.y), t(wl.obs))
    lib = N.lib()
    P = 8
    cost = gm.query_cost(t(wl.qx), t(wl.qy)).cpu().numpy()
    cuts = {"equal": [shard_range(wl.qx.size, r, P)[0] for r in range(P)] + [wl.qx.size], "cost": balanced_cuts(cost, P)}
    for name, c in cuts.items():
        for r in range(P):
            lo, hi = c[r], c[r + 1]
            qx, qy = t(wl.qx[lo:hi]), t(wl.qy[lo:hi])
            row = []
            for order in (1, 2):
                gm.set_option(N.SBO_OPT_QUERY_ORDER, order)
                for rep in range(3):
                    lib.sbo_profile(gm.ctx.handle, 1)
                    gm.tick(qx, qy, wl.beta, wl.f_min)
                    pm, pl, fm, fl = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_int64()
                    lib.sbo_profile_read(gm.ctx.handle, ctypes.byref(pm), ctypes.byref(pl), ctypes.byref(fm), ctypes.byref(fl))
                    w = ctypes.c_double()
                    lib.sbo_profile_work(gm.ctx.handle, ctypes.byref(w))
                row.append((pm.value, w.value / (2 * 256 * 128 * 64)))
            print(f"{name} r{r} [{lo},{hi}) m {hi - lo} (lo % {gw} = {lo % gw}): patches {row[0][0]:.2f} ms {row[0][1]:.4g} tiles"
                  f" | Morton {row[1][0]:.2f} ms {row[1][1]:.4g} tiles", flush=True)
    gm.set_option(N.SBO_OPT_QUERY_ORDER, 1)
    gm.close()


if __name__ == "__main__":
    main()
