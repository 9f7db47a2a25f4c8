"""Round 5: which probe query set tracks the whole grid's
fast-sweep variance error best.  For each calibration workload (the default
domain's data and path-shaped data, refitted with l in {0.2, 0.4, 0.8, 1.6}
and sn2 in {0.01, 0.1}) the fast (SBO_OPT_PRECISION 0) and precise (1) sweeps
run over the whole grid and over candidate probe sets; each set's normwise
variance error max|dv| / max v is compared with the whole grid's:
  cur     the library's probe: a 32 x 32 lattice over the data bounds + 512
          strided training locations (the k-d order's every (n/512)-th point)
  off     cur + the same 512 locations moved by l/2 (golden-angle directions)
  off4    cur + 512 locations moved by l/4
  off24   cur + 256 moved by l/4 and 256 by l/2
  lat64   a 64 x 64 lattice + the 512 training locations
and where the whole grid's worst point lies (its variance / the largest, its
distance to the nearest training point / l).  GPU diagnostic, one JSON line
per workload:  python tools/probe_design.py [n] [grid]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from scipy.spatial import cKDTree  # noqa: E402

from safe_bayesian_optimization_amd import TerrainMapper  # noqa: E402
from safe_bayesian_optimization_amd import _native as N  # noqa: E402
from safe_bayesian_optimization_amd.terrain import Hyper, path_workload, synthetic  # noqa: E402

GOLDEN = np.pi * (3.0 - np.sqrt(5.0))


def lattice(x, y, g):
    gx = np.linspace(x.min(), x.max(), g)
    gy = np.linspace(y.min(), y.max(), g)
    QY, QX = np.meshgrid(gy, gx, indexing="ij")
    return QX.reshape(-1), QY.reshape(-1)


def offset(px, py, d, phase=0):
    a = GOLDEN * (np.arange(px.size) + phase)
    return px + d * np.cos(a), py + d * np.sin(a)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    grid = int(sys.argv[2]) if len(sys.argv) > 2 else 500
    dev = torch.device("cuda:0")
    t = lambda a: torch.tensor(np.ascontiguousarray(a, np.float32), device=dev)  # noqa: E731

    def sweep(gm, qx, qy):
        v = []
        for prec in (0, 1):
            gm.set_option(N.SBO_OPT_PRECISION, prec)
            _, sd = gm.predict(t(qx), t(qy))
            torch.cuda.synchronize()
            v.append(sd.double().cpu().numpy() ** 2)
        gm.set_option(N.SBO_OPT_PRECISION, -1)
        return v

    def nerr(v):
        return float(np.abs(v[0] - v[1]).max() / max(v[1].max(), 1e-300))

    for data in ("syn", "path"):
        base = synthetic(n, grid, grid, seed=3) if data == "syn" else path_workload(n, grid, grid, seed=3)
        tree = cKDTree(np.stack([base.x, base.y], 1))
        for ell in (0.2, 0.4, 0.8, 1.6):
            for sn2 in (0.01, 0.1):
                gm = TerrainMapper(0, Hyper(length_scale=ell, noise_level=sn2))
                try:
                    gm.fit(t(base.x), t(base.y), t(base.obs))
                except N.SboError as ex:
                    print(json.dumps({"data": data, "l": ell, "sn2": sn2, "fit": str(ex)}), flush=True)
                    gm.close()
                    continue
                pi = gm.probe_info()
                o = gm.order()
                stride = max(n // 512, 1)
                sel = o[stride // 2::stride][:512]
                px, py = base.x[sel], base.y[sel]
                lx, ly = lattice(base.x, base.y, 32)
                sets = {
                    "cur": (np.r_[lx, px], np.r_[ly, py]),
                }
                for name, parts in (("off", [(0.5, 0)]), ("off4", [(0.25, 0)]), ("off24", [(0.25, 0), (0.5, 1)])):
                    qx, qy = [lx, px], [ly, py]
                    if len(parts) == 1:
                        ox, oy = offset(px, py, parts[0][0] * ell)
                        qx.append(ox)
                        qy.append(oy)
                    else:
                        for k, (d, ph) in enumerate(parts):
                            ox, oy = offset(px[k::2], py[k::2], d * ell, ph)
                            qx.append(ox)
                            qy.append(oy)
                    sets[name] = (np.concatenate(qx), np.concatenate(qy))
                l64x, l64y = lattice(base.x, base.y, 64)
                sets["lat64"] = (np.r_[l64x, px], np.r_[l64y, py])
                vw = sweep(gm, base.qx, base.qy)
                ew = nerr(vw)
                d = np.abs(vw[0] - vw[1])
                i = int(d.argmax())
                dist, _ = tree.query([base.qx[i], base.qy[i]])
                res = {"data": data, "n": n, "l": ell, "sn2": sn2, "precise_chosen": bool(pi["precise"]),
                       "lib_probe_err": pi["err"], "grid_err": ew,
                       "worst_var_over_max": float(vw[1][i] / vw[1].max()), "worst_dist_over_l": float(dist / ell)}
                for name, (qx, qy) in sets.items():
                    e = nerr(sweep(gm, qx, qy))
                    res[f"{name}_err"] = e
                    res[f"{name}_ratio"] = ew / max(e, 1e-30)
                print(json.dumps(res), flush=True)
                gm.close()


if __name__ == "__main__":
    main()
