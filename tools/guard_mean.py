"""Round 6: the inverse guard's two readings (variance err, mean err_mean) per
digit count against the whole-grid effect of the same inverse on the
posterior -- mu and var of the precise sweep (so the inverse's own effect
shows, not the fast sweep's budget) against the dgemm-inverse fit's, normwise
(max |d| / max |ref|).  Then the adaptive digits over three refits.
GPU diagnostic.
    python tools/guard_mean.py [workload ...]   (c4 box skip path cluster)"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from safe_bayesian_optimization_amd import TerrainMapper, synthetic  # noqa: E402
from safe_bayesian_optimization_amd import _native as N  # noqa: E402
from safe_bayesian_optimization_amd.terrain import clustered, path_workload, synthetic_box  # noqa: E402


WORKLOADS = {
    "c4": lambda: synthetic(16384, 300, 300, seed=0),
    "box": lambda: synthetic_box(16384, 300, 120, seed=0),
    "skip": lambda: synthetic(8192, 200, 160, seed=21),
    "path": lambda: path_workload(16384, 300, seed=0),
    "cluster": lambda: clustered(16384, 300, 300, seed=7),
}


def main():
    names = sys.argv[1:] or list(WORKLOADS)
    dev = torch.device("cuda:0")
    t = lambda a: torch.tensor(np.ascontiguousarray(a, np.float32), device=dev)  # noqa: E731
    for name in names:
        wl = WORKLOADS[name]()
        X, Y, O, QX, QY = t(wl.x), t(wl.y), t(wl.obs), t(wl.qx), t(wl.qy)
        ref = None
        for oz in (0, 6, 5, 4):
            gm = TerrainMapper(0, wl.hyper)
            gm.set_option(N.SBO_OPT_PRECISION, 1)
            gm.set_option(N.SBO_OPT_INV_OZ, oz)
            gm.set_option(N.SBO_OPT_INV_OZ_ADAPT, 0)
            gm.set_option(N.SBO_OPT_INV_CHECK, 2 if oz == 0 else 0)   # (guard off: keep the sliced inverse)
            gm.fit(X, Y, O)
            mu, sd = gm.predict(QX, QY)
            mu = mu.cpu().numpy().astype(np.float64)
            var = sd.cpu().numpy().astype(np.float64) ** 2
            # the guard's readings of this very inverse: refit with the guard on
            # (the same data and digits give the same inverse)
            gm.set_option(N.SBO_OPT_INV_CHECK, 2)
            gm.set_option(N.SBO_OPT_INV_OZ, oz)
            gm.set_option(N.SBO_OPT_INV_OZ_ADAPT, 0)
            gm.fit(X, Y, O)
            c = gm.inverse_check()
            line = (f"{name} N={wl.x.size} digits={c['digits']}: guard var {c['err']:.2e} mean {c['err_mean']:.2e} "
                    f"fired {c['fired']} kept {c['kept_digits']} ({c['ms']:.2f} ms)")
            if ref is None:
                ref = (mu, var)
            else:
                dm = np.abs(mu - ref[0]).max() / np.abs(ref[0]).max()
                dv = np.abs(var - ref[1]).max() / np.abs(ref[1]).max()
                line += f" || grid vs dgemm: mu {dm:.2e} var {dv:.2e}"
            print(line, flush=True)
            gm.close()
        gm = TerrainMapper(0, wl.hyper)
        fits = []
        for _ in range(4):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            gm.fit(X, Y, O)
            torch.cuda.synchronize()
            c = gm.inverse_check()
            fits.append(f"{(time.perf_counter() - t0) * 1e3:.1f} ms d{c['digits']} v{c['err']:.1e} m{c['err_mean']:.1e}"
                        + (f" FIRED->d{c['kept_digits']}" if c['fired'] else ""))
        print(f"{name} adapt: " + " | ".join(fits), flush=True)
        gm.close()


if __name__ == "__main__":
    main()
