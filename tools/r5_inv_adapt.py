"""Round 5: the sliced inverse's digits per fit (SBO_OPT_INV_OZ_ADAPT) against
fixed digits and dgemm products: warm fit times, the guard's digits / measure
per fit, and the posterior over the whole grid against the dgemm fit's
(normwise max |d| / max |ref| of mu and of var).  GPU diagnostic.
PREC=1 forces the precise sweep (the inverse's own effect, without the fast
sweep's error budget).
    python tools/r5_inv_adapt.py [n ...]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from safe_bayesian_optimization_amd import TerrainMapper, synthetic  # noqa: E402
from safe_bayesian_optimization_amd import _native as N  # noqa: E402
from safe_bayesian_optimization_amd.terrain import synthetic_box  # noqa: E402


def main():
    ns = [int(v) for v in sys.argv[1:]] or [16384]
    dev = torch.device("cuda:0")
    t = lambda a: torch.tensor(np.ascontiguousarray(a, np.float32), device=dev)  # noqa: E731
    for n in ns:
        wls = (("synthetic", synthetic(n, 1000, 1000, seed=0)), ("lpsc box", synthetic_box(n, 1000, 1000, seed=0)))
        for name, wl in wls[:int(os.environ.get("WLS", "2"))]:
            ref = None
            for oz, adapt in ((0, 0), (6, 0), (5, 0), (4, 0), (6, 1)):
                gm = TerrainMapper(0, wl.hyper)
                if os.environ.get("PREC"):
                    gm.set_option(N.SBO_OPT_PRECISION, int(os.environ["PREC"]))
                gm.set_option(N.SBO_OPT_INV_OZ, oz)
                gm.set_option(N.SBO_OPT_INV_OZ_ADAPT, adapt)
                X, Y, O = t(wl.x), t(wl.y), t(wl.obs)
                fits = []
                for _ in range(5):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    gm.fit(X, Y, O)
                    torch.cuda.synchronize()
                    c = gm.inverse_check()
                    fits.append(f"{(time.perf_counter() - t0) * 1e3:.1f} ms d{c['digits']} {c['err']:.1e}"
                                + (" FIRED" if c['fired'] else ""))
                precise, perr, _, _ = gm.precision()
                mu, sd = gm.predict(t(wl.qx), t(wl.qy))
                mu = mu.cpu().numpy().astype(np.float64)
                var = sd.cpu().numpy().astype(np.float64) ** 2
                line = f"{name} N={n} inv_oz={oz} adapt={adapt} precise={precise}: " + " | ".join(fits)
                if ref is None:
                    ref = (mu, var)
                else:
                    dm = np.abs(mu - ref[0]).max() / np.abs(ref[0]).max()
                    dv = np.abs(var - ref[1]).max() / np.abs(ref[1]).max()
                    line += f" || vs dgemm: mu {dm:.2e} var {dv:.2e}"
                print(line, flush=True)
                gm.close()


if __name__ == "__main__":
    main()
