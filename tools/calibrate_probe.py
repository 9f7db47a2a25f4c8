"""Round 5: calibrate the precision probe and
the inverse guard over hyper-parameters.  For each workload (the default
domain's data and the path-shaped data, refitted with l in {0.2, 0.4, 0.8,
1.6} and sn2 in {0.01, 0.1}; the data are generated with the default
hyper-parameters, so a longer l packs more points per l^2):
  - fit with default options: the probe's numbers (sbo_get_probe) and the
    guard's (sbo_get_inverse_check);
  - the fast sweep (SBO_OPT_PRECISION 0) and the precise one (1) over the whole
    grid on that fit: the fast sweep's normwise variance error against the
    precise one, and its ratio to the probe's error (the probe threshold
    5e-6 times the largest ratio must stay under the 1e-5 contract);
  - the same fit with dgemm products in the inverse (SBO_OPT_INV_OZ 0), the
    precise sweep over the whole grid: the sliced inverse's own effect on the
    variance, and its ratio to the guard's measure (the guard's 5e-7 times the
    largest ratio must stay far under the contract).
GPU diagnostic, one JSON line per workload:
    python tools/calibrate_probe.py [n] [grid]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from safe_bayesian_optimization_amd import TerrainMapper  # noqa: E402
from safe_bayesian_optimization_amd import _native as N  # noqa: E402
from safe_bayesian_optimization_amd.terrain import Hyper, path_workload, synthetic  # noqa: E402


def nrel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


PROBE_SIZES = [(48, 1024), (64, 2048)]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    grid = int(sys.argv[2]) if len(sys.argv) > 2 else 500
    dev = torch.device("cuda:0")
    t = lambda a: torch.tensor(np.ascontiguousarray(a, np.float32), device=dev)  # noqa: E731
    for data in ("syn", "path"):
        base = synthetic(n, grid, grid, seed=3) if data == "syn" else path_workload(n, grid, grid, seed=3)
        for ell in (0.2, 0.4, 0.8, 1.6):
            for sn2 in (0.01, 0.1):
                h = Hyper(length_scale=ell, noise_level=sn2)
                gm = TerrainMapper(0, h)
                try:
                    gm.fit(t(base.x), t(base.y), t(base.obs))
                except N.SboError as ex:   # NOT_SPD: the f32 factor fails (reported, not calibrated)
                    print(json.dumps({"data": data, "n": n, "l": ell, "sn2": sn2, "fit": str(ex)}), flush=True)
                    gm.close()
                    continue
                pi = gm.probe_info()
                chk = gm.inverse_check()
                # the probe at other sizes on the same data (SBO_OPT_PROBE_SIZE: grid side, training points)
                probe_sizes, fit_ms = {}, {}
                X, Y, OB = t(base.x), t(base.y), t(base.obs)
                for pg, pt in [(32, 512)] + PROBE_SIZES:
                    gm.set_option(N.SBO_OPT_PROBE_SIZE, (pg << 16) | pt)
                    gm.fit(X, Y, OB)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    gm.fit(X, Y, OB)
                    torch.cuda.synchronize()
                    fit_ms[f"{pg}x{pg}+{pt}"] = (time.perf_counter() - t0) * 1e3
                    probe_sizes[f"{pg}x{pg}+{pt}"] = gm.probe_info()["err"]
                gm.set_option(N.SBO_OPT_PROBE_SIZE, (32 << 16) | 512)
                gm.fit(X, Y, OB)
                qx, qy = t(base.qx), t(base.qy)
                v = {}
                for prec in (0, 1):
                    gm.set_option(N.SBO_OPT_PRECISION, prec)
                    mu, sd = gm.predict(qx, qy)
                    torch.cuda.synchronize()
                    v[prec] = sd.double().cpu().numpy() ** 2
                gm.set_option(N.SBO_OPT_PRECISION, -1)
                err_fast = nrel(v[0], v[1])
                # the inverse with dgemm products: the sliced inverse's own effect
                gm.set_option(N.SBO_OPT_INV_OZ, 0)
                gm.fit(t(base.x), t(base.y), t(base.obs))
                gm.set_option(N.SBO_OPT_PRECISION, 1)
                _, sd0 = gm.predict(qx, qy)
                torch.cuda.synchronize()
                v0 = sd0.double().cpu().numpy() ** 2
                inv_eff = nrel(v[1], v0)
                res = {"data": data, "n": n, "m": int(base.qx.size), "l": ell, "sn2": sn2,
                       "precise_chosen": bool(pi["precise"]), "probe_err": pi["err"],
                       "fast_vs_precise_whole_grid_var": err_fast,
                       "ratio_grid_over_probe": err_fast / max(pi["err"], 1e-30),
                       "guard_ran": chk["ran"], "guard_err": chk["err"], "guard_fired": chk["fired"],
                       "guard_ms": chk["ms"],
                       "sliced_vs_dgemm_whole_grid_var": inv_eff,
                       "ratio_grid_over_guard": inv_eff / max(chk["err"], 1e-30) if chk["ran"] else None,
                       "grid_var_min": float(v[1].min()), "grid_var_max": float(v[1].max()),
                       "probe_err_by_size": probe_sizes, "fit_ms_by_probe_size": fit_ms,
                       "ratio_by_probe_size": {k: err_fast / max(e, 1e-30) for k, e in probe_sizes.items()}}
                print(json.dumps(res), flush=True)
                gm.close()


if __name__ == "__main__":
    main()
