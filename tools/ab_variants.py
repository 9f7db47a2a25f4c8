"""Interleaved A/B of predictive-kernel variants in ONE process (guide rule 24).

  python tools/ab_variants.py --config C4 --variants 0 1 --rounds 3 [--opt NAME=VAL ...]
Prints the median predict-kernel time per variant and the max |d| of mu/sd vs variant 0."""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="C4")
    p.add_argument("--variants", type=int, nargs="+", default=[0, 1])
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--opt", nargs="*", default=[])
    p.add_argument("--box", action="store_true", help="the config's N and grid on the lpsc.yaml box (stress variant)")
    a = p.parse_args()
    import torch
    from safe_bayesian_optimization_amd import TerrainMapper, synthetic
    from safe_bayesian_optimization_amd import _native as N
    from safe_bayesian_optimization_amd.terrain import CONFIGS, synthetic_box
    n, gw, gh = CONFIGS[a.config]
    wl = synthetic_box(n, gw, gh, seed=0) if a.box else synthetic(n, gw, gh, seed=0)
    dev = torch.device("cuda:0")
    t = lambda v: torch.as_tensor(np.ascontiguousarray(v, np.float32), device=dev)  # noqa: E731
    gm = TerrainMapper(0, wl.hyper)
    for kv in a.opt:
        k, v = kv.split("=")
        gm.set_option(getattr(N, k), int(v))
    gm.fit(t(wl.x), t(wl.y), t(wl.obs))
    qx, qy = t(wl.qx), t(wl.qy)
    m = qx.numel()
    lib = N.lib()
    times = {v: [] for v in a.variants}
    outs = {}
    for r in range(a.rounds + 1):
        for v in a.variants:
            gm.set_option(N.SBO_OPT_KERNEL_VARIANT, v)
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
            if r > 0:
                times[v].append((pm.value, w.value / (pm.value * 1e-3) / 1e12, w.value, mf.value, list(lv)))
            outs[v] = (mu.cpu().numpy(), sd.cpu().numpy())
    for v in a.variants:
        ms = np.median([x[0] for x in times[v]])
        tf = np.median([x[1] for x in times[v]])
        dmu = np.abs(outs[v][0] - outs[a.variants[0]][0]).max()
        dsd = np.abs(outs[v][1] - outs[a.variants[0]][1]).max()
        fl, mf = times[v][-1][2], times[v][-1][3]
        print(f"variant {v}: {ms:.2f} ms  {tf:.1f} TF exec  tiles {fl / (2 * 256 * 128 * 64):.4g}  MFMA products/tile "
              f"{mf / max(fl, 1.0):.3f} levels {times[v][-1][4]}  | max|dmu| {dmu:.2e} max|dsd| {dsd:.2e}", flush=True)


if __name__ == "__main__":
    main()
