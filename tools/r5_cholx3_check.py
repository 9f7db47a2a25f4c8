"""Round 5: SBO_OPT_CHOL_GEMM 3 (the Cholesky's outer-panel updates on the
bf16 matrix cores with split operands) against 0 (rocBLAS) at C4 and on the
lpsc box: the factors' largest difference relative to the largest entry, and
the posterior of both fits over the whole grid (normwise max |d| / max |ref|
of mu and var).  GPU diagnostic: python tools/r5_cholx3_check.py [n]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from safe_bayesian_optimization_amd import TerrainMapper, synthetic  # noqa: E402
from safe_bayesian_optimization_amd import _native as N  # noqa: E402
from safe_bayesian_optimization_amd.terrain import synthetic_box  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    dev = torch.device("cuda:0")
    t = lambda a: torch.tensor(np.ascontiguousarray(a, np.float32), device=dev)  # noqa: E731
    for name, wl in (("C4", synthetic(n, 1000, 1000, seed=0)), ("lpsc box", synthetic_box(n, 1000, 1000, seed=0))):
        out = {}
        for g in (0, 3):
            gm = TerrainMapper(0, wl.hyper)
            gm.set_option(N.SBO_OPT_CHOL_GEMM, g)
            gm.fit(t(wl.x), t(wl.y), t(wl.obs))
            L, _ = gm.factor()
            mu, sd = gm.predict(t(wl.qx), t(wl.qy))
            out[g] = (L, mu.cpu().numpy().astype(np.float64), sd.cpu().numpy().astype(np.float64) ** 2,
                      gm.precision()[0])
            gm.close()
        L0, L3 = out[0][0], out[3][0]
        dl = float(np.abs(L0.astype(np.float64) - L3).max() / np.abs(L0).max())
        dm = float(np.abs(out[3][1] - out[0][1]).max() / np.abs(out[0][1]).max())
        dv = float(np.abs(out[3][2] - out[0][2]).max() / np.abs(out[0][2]).max())
        print(f"{name} N={n}: factor max diff {dl:.2e} of max |L|; posterior mu {dm:.2e} var {dv:.2e} "
              f"(precise sweep: {out[0][3]} / {out[3][3]})", flush=True)


if __name__ == "__main__":
    main()
