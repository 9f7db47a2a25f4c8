"""The fit-time precision probe (SBO_OPT_PRECISION = -1) on every bench
workload: the fast sweep's variance error on the 32 x 32 probe grid, the
probe's variance range, the decision, and the warm fit time with and without
the probe (GPU diagnostic, one JSON line per workload)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from safe_bayesian_optimization_amd import TerrainMapper, synthetic  # noqa: E402
from safe_bayesian_optimization_amd import _native as N  # noqa: E402
from safe_bayesian_optimization_amd.terrain import CONFIGS, synthetic_box  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a, np.float32), device=dev)  # noqa: E731
    cases = [(c, synthetic(*CONFIGS[c], seed=0)) for c in ("C2", "C3", "C4")]
    cases += [("C5-final", synthetic(8000, 512, 512, seed=0)), ("lpsc-box-16384", synthetic_box(16384, 1000, 1000, seed=0)),
              ("lpsc-box-4096", synthetic_box(4096, 300, 120, seed=0)), ("lpsc-box-1024", synthetic_box(1024, 300, 120, seed=0))]
    for name, wl in cases:
        gm = TerrainMapper(0, wl.hyper)
        X, Y, O = t(wl.x), t(wl.y), t(wl.obs)
        gm.fit(X, Y, O)
        res = {"workload": name, "n": int(wl.x.size)}
        for opt in (-1, 0):
            gm.set_option(N.SBO_OPT_PRECISION, opt)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            gm.fit(X, Y, O)
            torch.cuda.synchronize()
            res[f"fit_ms_opt{opt}"] = (time.perf_counter() - t0) * 1e3
        gm.set_option(N.SBO_OPT_PRECISION, -1)
        p, e, vmin, vmax = gm.precision()
        res.update(precise=p, probe_err=e, probe_var_min=vmin, probe_var_max=vmax)
        # tick time both ways on the workload's grid
        qx, qy = t(wl.qx), t(wl.qy)
        for opt in (1, 0):
            gm.set_option(N.SBO_OPT_PRECISION, opt)
            gm.tick(qx, qy, wl.beta, wl.f_min)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                gm.tick(qx, qy, wl.beta, wl.f_min)
            torch.cuda.synchronize()
            res[f"tick_ms_{'precise' if opt else 'fast'}"] = (time.perf_counter() - t0) * 1e3 / 3
        print(json.dumps(res), flush=True)
        gm.close()


if __name__ == "__main__":
    main()
