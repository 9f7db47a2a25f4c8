"""A/B of the fit's f64 inverse with its top-level products by rocBLAS dgemm
(SBO_OPT_INV_OZ 0) or by the int8-sliced GEMM (5 / 6 digits,
csrc/ozgemm.hip): warm fit time, the precision probe's verdict and error,
and the posterior over the whole grid against the dgemm fit's (normwise
max |d| / max |ref| of mu and of var).  Workloads: C4 (synthetic, N = 16384,
1000 x 1000) and the lpsc box (N = 16384, 1000 x 1000).  INV_OZ_MIN (round
5): the smallest sliced splits to try (SBO_OPT_INV_OZ_MIN, default "4096");
the guard's measure (sbo_get_inverse_check) is printed.  GPU diagnostic.
    python tools/inv_oz_ab.py [n] [digits ...]"""
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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    digits = [int(v) for v in sys.argv[2:]] or [6, 5]
    dev = torch.device("cuda:0")
    t = lambda a: torch.tensor(np.ascontiguousarray(a, np.float32), device=dev)  # noqa: E731
    for name, wl in (("C4", synthetic(n, 1000, 1000, seed=0)), ("lpsc box", synthetic_box(n, 1000, 1000, seed=0))):
        ref = None
        mins = [int(v) for v in os.environ.get("INV_OZ_MIN", "4096").split()]
        for oz, omin in [(0, 4096)] + [(d, m) for d in digits for m in mins]:
            gm = TerrainMapper(0, wl.hyper)
            gm.set_option(N.SBO_OPT_INV_OZ, oz)
            gm.set_option(N.SBO_OPT_INV_OZ_MIN, omin)
            X, Y, O = t(wl.x), t(wl.y), t(wl.obs)
            ts = []
            for _ in range(4):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                gm.fit(X, Y, O)
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t0) * 1e3)
            precise, perr, vmin, vmax = gm.precision()
            mu, sd = gm.predict(t(wl.qx), t(wl.qy))
            mu = mu.cpu().numpy().astype(np.float64)
            var = sd.cpu().numpy().astype(np.float64) ** 2
            chk = gm.inverse_check()
            line = (f"{name} N={n} inv_oz={oz} min={omin}: warm fits {', '.join(f'{v:.1f}' for v in ts[1:])} ms, "
                    f"precise={precise} probe_err={perr:.3e} guard ran={chk['ran']} err={chk['err']:.2e} "
                    f"fired={chk['fired']} {chk['ms']:.2f} ms")
            if ref is None:
                ref = (mu, var)
            else:
                dm = np.abs(mu - ref[0]).max() / np.abs(ref[0]).max()
                dv = np.abs(var - ref[1]).max() / np.abs(ref[1]).max()
                line += f", vs dgemm fit: mu {dm:.3e} var {dv:.3e}"
            print(line, flush=True)
            gm.close()


if __name__ == "__main__":
    main()
