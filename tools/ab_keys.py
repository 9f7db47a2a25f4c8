"""Interleaved A/B of the precision-level rank keys (SBO_LVL_KEYS, tuning) in one process.

  python tools/ab_keys.py --config C4 --keys 0.8,1.72 0,0 1.6,3.4 --rounds 2
Prints the median predict-kernel time, the tiles per level and max |d sd| vs the first key pair."""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="C4")
    p.add_argument("--keys", nargs="+", default=["0.8,1.72"])
    p.add_argument("--rounds", type=int, default=2)
    p.add_argument("--variant", type=int, default=3)
    a = p.parse_args()
    import torch
    from safe_bayesian_optimization_amd import TerrainMapper, synthetic
    from safe_bayesian_optimization_amd import _native as N
    from safe_bayesian_optimization_amd.terrain import CONFIGS
    n, gw, gh = CONFIGS[a.config]
    wl = synthetic(n, gw, gh, seed=0)
    dev = torch.device("cuda:0")
    t = lambda v: torch.as_tensor(np.ascontiguousarray(v, np.float32), device=dev)  # noqa: E731
    gm = TerrainMapper(0, wl.hyper)
    gm.set_option(N.SBO_OPT_KERNEL_VARIANT, a.variant)
    gm.fit(t(wl.x), t(wl.y), t(wl.obs))
    qx, qy = t(wl.qx), t(wl.qy)
    m = qx.numel()
    lib = N.lib()
    res = {k: [] for k in a.keys}
    outs = {}
    for r in range(a.rounds + 1):
        for k in a.keys:
            os.environ["SBO_LVL_KEYS"] = k.replace("m", "-")
            sd = torch.empty(m, device=dev)
            lib.sbo_profile(gm.ctx.handle, 1)
            gm.tick(qx, qy, wl.beta, wl.f_min, outputs=dict(sd=sd))
            pm, pl, fm, fl = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_int64()
            lib.sbo_profile_read(gm.ctx.handle, ctypes.byref(pm), ctypes.byref(pl), ctypes.byref(fm), ctypes.byref(fl))
            mf = ctypes.c_double()
            lv = (ctypes.c_int64 * 3)()
            lib.sbo_profile_mfma(gm.ctx.handle, ctypes.byref(mf), lv)
            if r > 0:
                res[k].append((pm.value, list(lv)))
            outs[k] = sd.cpu().numpy()
    for k in a.keys:
        ms = np.median([x[0] for x in res[k]])
        d = np.abs(outs[k].astype(np.float64) ** 2 - outs[a.keys[0]].astype(np.float64) ** 2).max()
        print(f"keys {k}: {ms:.2f} ms  levels {res[k][-1][1]}  max|d var| vs first {d:.2e}", flush=True)


if __name__ == "__main__":
    main()
