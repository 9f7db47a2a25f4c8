"""Round 5: the C2 fit (N = 2048, 256 x 256) under the precision probe's
options -- the precise kernel its reference sweep uses, its size, or no
probe -- median warm fit and the probe's verdict.  GPU diagnostic.
    python tools/r5_c2_probe.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from safe_bayesian_optimization_amd import TerrainMapper, synthetic  # noqa: E402
from safe_bayesian_optimization_amd import _native as N  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    wl = synthetic(2048, 256, 256, seed=0)
    t = lambda a: torch.tensor(np.ascontiguousarray(a, np.float32), device=dev)  # noqa: E731
    X, Y, O = t(wl.x), t(wl.y), t(wl.obs)
    variants = [("default", {}), ("precise kernel 0", {N.SBO_OPT_PRECISE_KERNEL: 0}),
                ("precise kernel 1", {N.SBO_OPT_PRECISE_KERNEL: 1}),
                ("precise kernel 4", {N.SBO_OPT_PRECISE_KERNEL: 4}),
                ("probe 16^2 + 256", {N.SBO_OPT_PROBE_SIZE: 16 << 16 | 256}),
                ("probe 32^2 + 256", {N.SBO_OPT_PROBE_SIZE: 32 << 16 | 256}),
                ("probe 16^2 + 512", {N.SBO_OPT_PROBE_SIZE: 16 << 16 | 512}),
                ("no probe", {N.SBO_OPT_PRECISION: 0})]
    for name, opts in variants:
        gm = TerrainMapper(0, wl.hyper)
        for k, v in opts.items():
            gm.set_option(k, v)
        ts = []
        for _ in range(12):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            gm.fit(X, Y, O)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        precise, perr, vmin, vmax = gm.precision()
        print(f"C2 {name}: warm fit median {np.median(ts[2:]):.2f} ms (min {min(ts[2:]):.2f}); precise={precise} "
              f"probe err {perr:.2e}", flush=True)
        gm.close()


if __name__ == "__main__":
    main()
