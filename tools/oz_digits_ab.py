"""Precise sweep A/B on the lpsc box (config/lpsc.yaml:32-37): tick time and
the variance / mean error against the fp64 oracle given the device factor, for
the library named by SBO_LIB (run once per build).
    SBO_LIB=... python tools/oz_digits_ab.py [N] [ticks]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from oracle import oracle as O  # noqa: E402
from safe_bayesian_optimization_amd import TerrainMapper  # noqa: E402
from safe_bayesian_optimization_amd.terrain import synthetic_box  # noqa: E402


def f32(a):
    return np.ascontiguousarray(a, np.float32)


def nrel(a, b):
    return float(np.abs(np.asarray(a, np.float64) - b).max() / max(np.abs(b).max(), 1e-30))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    ticks = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda:0")
    O.set_threads(16)
    wl = synthetic_box(n, 1000, 1000, seed=0)
    h = wl.hyper
    gm = TerrainMapper(0, h)
    t = lambda a: torch.tensor(f32(a), device=dev)  # noqa: E731
    gm.fit(t(wl.x), t(wl.y), t(wl.obs))
    qx, qy = t(wl.qx), t(wl.qy)
    mu, sd = gm.predict(qx, qy)
    torch.cuda.synchronize()
    ts = []
    for _ in range(ticks):
        t0 = time.perf_counter()
        mu, sd = gm.predict(qx, qy)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    mu, sd = mu.cpu().numpy(), sd.cpu().numpy()
    m = wl.qx.size
    sel = np.sort(np.random.default_rng(7).choice(m, 2048, replace=False))
    L, alpha = gm.factor()
    o = gm.order()
    xs, ys = f32(wl.x)[o], f32(wl.y)[o]
    Lcm = O.colmajor_from_lower(L.astype(np.float64))
    omu, ovar = O.predict(Lcm, alpha.astype(np.float64), xs, ys, f32(wl.qx[sel]), f32(wl.qy[sel]),
                          h.length_scale, h.sf2, h.prior_mean)
    print(json.dumps({"lib": os.environ.get("SBO_LIB", "libsbo.so"), "n": n, "precise": gm.precision()[0]
                      if hasattr(gm, "precision") else None, "tick_ms": ts,
                      "var": nrel(sd[sel].astype(np.float64) ** 2, ovar), "mu": nrel(mu[sel], omu)}), flush=True)
    gm.close()


if __name__ == "__main__":
    main()
