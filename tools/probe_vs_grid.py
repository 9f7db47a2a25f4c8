"""The precision probe against the whole grid (DESIGN.md 5a
records the probe-vs-full-grid ratio on every workload).  For each workload:
fit with default options, the probe's numbers (sbo_get_probe), then the fast
sweep (SBO_OPT_PRECISION 0) and the precise sweep (1) over the workload's whole
grid on the same fit; the fast sweep's normwise variance error against the
precise one over the whole grid, and its ratio to the probe's error.  GPU
diagnostic (tools/), one JSON line per workload.
    python tools/probe_vs_grid.py [names...]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from safe_bayesian_optimization_amd import TerrainMapper  # noqa: E402
from safe_bayesian_optimization_amd import _native as N  # noqa: E402
from safe_bayesian_optimization_amd.terrain import path_workload, synthetic, synthetic_box  # noqa: E402

WORKLOADS = {
    "C2": lambda: synthetic(2048, 256, 256, seed=0, name="C2"),
    "C3": lambda: synthetic(8192, 1024, 1024, seed=0, name="C3"),
    "C4": lambda: synthetic(16384, 1000, 1000, seed=0, name="C4"),
    "C5_last": lambda: synthetic(8000, 512, 512, seed=0, name="C5 (all 8000 points)"),
    "path": lambda: path_workload(16384, 1000, 1000, seed=0),
    "path_8k": lambda: path_workload(8192, 1000, 1000, seed=1),
    "lpsc_4096": lambda: synthetic_box(4096, 300, 120, seed=0),
    "lpsc_1024": lambda: synthetic_box(1024, 300, 120, seed=0),
}


def main():
    names = sys.argv[1:] or list(WORKLOADS)
    dev = torch.device("cuda:0")
    for name in names:
        wl = WORKLOADS[name]()
        gm = TerrainMapper(0, wl.hyper)
        t = lambda a: torch.tensor(np.ascontiguousarray(a, np.float32), device=dev)  # noqa: E731
        gm.fit(t(wl.x), t(wl.y), t(wl.obs))
        pi = gm.probe_info()
        qx, qy = t(wl.qx), t(wl.qy)
        out = {}
        for prec in (0, 1):
            gm.set_option(N.SBO_OPT_PRECISION, prec)
            mu, sd = gm.predict(qx, qy)
            torch.cuda.synchronize()
            out[prec] = (mu.double().cpu().numpy(), sd.double().cpu().numpy() ** 2)
        gm.set_option(N.SBO_OPT_PRECISION, -1)
        vf, vp = out[0][1], out[1][1]
        err = float(np.abs(vf - vp).max() / np.abs(vp).max())
        res = {"workload": name, "n": int(wl.x.size), "m": int(wl.qx.size), "precise_chosen": bool(pi["precise"]),
               "probe_err": pi["err"], "probe_err_grid": pi["err_grid"], "probe_err_train": pi["err_train"],
               "probe_var_max": pi["var_max"], "grid_var_max": float(vp.max()), "grid_var_min": float(vp.min()),
               "fast_vs_precise_whole_grid_var": err, "ratio_grid_over_probe": err / max(pi["err"], 1e-30),
               "fast_vs_precise_whole_grid_mu": float(np.abs(out[0][0] - out[1][0]).max()
                                                      / np.abs(out[1][0]).max())}
        print(json.dumps(res), flush=True)
        gm.close()


if __name__ == "__main__":
    main()
