"""Fit once and run K planning ticks on cuda:0 (profiling driver for rocprofv3)."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="C2")
    p.add_argument("--n", type=int)
    p.add_argument("--grid", type=int)
    p.add_argument("--ticks", type=int, default=3)
    p.add_argument("--opt", nargs="*", default=[], help="NAME=VALUE library options (e.g. SBO_OPT_TILE_SKIP=0)")
    p.add_argument("--box", action="store_true", help="the lpsc.yaml stress box [0,1] x [0,2.5] (SURVEY 8(d))")
    a = p.parse_args()
    import torch
    from safe_bayesian_optimization_amd import TerrainMapper, synthetic
    from safe_bayesian_optimization_amd.terrain import CONFIGS
    if a.config == "C5":
        return streaming(a)
    n, gw, gh = CONFIGS[a.config]
    n = a.n or n
    if a.grid:
        gw = gh = a.grid
    if a.box:
        from safe_bayesian_optimization_amd.terrain import synthetic_box
        wl = synthetic_box(n, gw, gh, seed=0)
    else:
        wl = synthetic(n, gw, gh, seed=0)
    dev = torch.device("cuda:0")
    t = lambda v: torch.as_tensor(np.ascontiguousarray(v, np.float32), device=dev)  # noqa: E731
    gm = TerrainMapper(0, wl.hyper)
    from safe_bayesian_optimization_amd import _native as N
    for kv in a.opt:
        k, v = kv.split("=")
        gm.set_option(getattr(N, k), int(v))
    gm.fit(t(wl.x), t(wl.y), t(wl.obs))
    qx, qy = t(wl.qx), t(wl.qy)
    m = qx.numel()
    outs = dict(mu=torch.empty(m, device=dev), sd=torch.empty(m, device=dev),
                lo=torch.empty(m, dtype=torch.float64, device=dev), hi=torch.empty(m, dtype=torch.float64, device=dev),
                safe=torch.empty(m, dtype=torch.uint8, device=dev))
    for _ in range(a.ticks):
        gm.tick(qx, qy, wl.beta, wl.f_min, outputs=outs)
    torch.cuda.synchronize()
    print("done", n, m)


def streaming(a):
    """C5 as bench.py runs it: fit 1000 points, 50 appends to 8000, a 512 x 512
    tick after each (so per-kernel PMC averages match the bench's launches)."""
    import torch
    from safe_bayesian_optimization_amd import TerrainMapper, synthetic
    from safe_bayesian_optimization_amd import _native as N
    n_end, n0, iters, g = 8000, 1000, 50, a.grid or 512
    wl = synthetic(n_end, g, g, seed=0, name="C5")
    chunks = np.linspace(n0, n_end, iters + 1).round().astype(int)
    dev = torch.device("cuda:0")
    t = lambda v: torch.as_tensor(np.ascontiguousarray(v, np.float32), device=dev)  # noqa: E731
    X, Y, OBS = t(wl.x), t(wl.y), t(wl.obs)
    qx, qy = t(wl.qx), t(wl.qy)
    m = qx.numel()
    gm = TerrainMapper(0, wl.hyper)
    for kv in a.opt:
        k, v = kv.split("=")
        gm.set_option(getattr(N, k), int(v))
    outs = dict(mu=torch.empty(m, device=dev), sd=torch.empty(m, device=dev),
                lo=torch.empty(m, dtype=torch.float64, device=dev), hi=torch.empty(m, dtype=torch.float64, device=dev),
                safe=torch.empty(m, dtype=torch.uint8, device=dev))
    gm.fit(X[:n0], Y[:n0], OBS[:n0])
    for i in range(iters):
        gm.append(X[chunks[i]:chunks[i + 1]], Y[chunks[i]:chunks[i + 1]], OBS[chunks[i]:chunks[i + 1]])
        gm.tick(qx, qy, wl.beta, wl.f_min, outputs=outs)
    torch.cuda.synchronize()
    print("done C5", gm.n, m)


if __name__ == "__main__":
    main()
