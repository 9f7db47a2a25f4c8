"""Generate the committed golden fixtures under tests/golden/.

The reference ships no tests, fixtures or golden vectors for this path
 and its GP half lives in an external package that is not
under /root/reference.  These fixtures therefore come from two
INDEPENDENT implementations of the GP math contract:

  * numpy/scipy fp64 (explicit K, cho_factor/cho_solve, solve_triangular);
  * scikit-learn GaussianProcessRegressor with
    ConstantKernel(sf2,'fixed')*RBF(l,'fixed') + WhiteKernel(sn2,'fixed'),
    optimizer=None (its std includes the white noise: subtract sn2).

The script asserts the two agree before writing anything.  The acquisition
fields (lo/hi/safe) restate node.cpp:409-416 with plain numpy float64 ops.
Contour fixtures are hand-derived from OpenCV 4.5.x's RETR_EXTERNAL /
CHAIN_APPROX_NONE border follower (see oracle/sbo_oracle.c) and written as
literals below.

Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import scipy.linalg as sla

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from safe_bayesian_optimization_amd import terrain as T  # noqa: E402  (pure numpy)


def gp_numpy(x, y, obs, qx, qy, h: T.Hyper):
    X = np.c_[x, y]
    Q = np.c_[qx, qy]
    d2 = ((X[:, None, :] - X[None, :, :]) ** 2).sum(-1)
    K = h.sf2 * np.exp(-d2 / (2 * h.length_scale ** 2)) + h.sn2 * np.eye(len(x))
    c, low = sla.cho_factor(K, lower=True)
    alpha = sla.cho_solve((c, low), obs - h.prior_mean)
    d2q = ((Q[:, None, :] - X[None, :, :]) ** 2).sum(-1)
    Ks = h.sf2 * np.exp(-d2q / (2 * h.length_scale ** 2))
    mu = h.prior_mean + Ks @ alpha
    V = sla.solve_triangular(np.tril(c), Ks.T, lower=True)
    var = np.maximum(h.sf2 - (V * V).sum(0), 0.0)
    return mu, var


def gp_sklearn(x, y, obs, qx, qy, h: T.Hyper):
    from sklearn.gaussian_process import GaussianProcessRegressor
    from sklearn.gaussian_process.kernels import RBF, ConstantKernel, WhiteKernel
    k = ConstantKernel(h.sf2, "fixed") * RBF(h.length_scale, "fixed") + WhiteKernel(h.sn2, "fixed")
    g = GaussianProcessRegressor(k, optimizer=None, normalize_y=False)
    g.fit(np.c_[x, y], obs - h.prior_mean)
    mu, sd = g.predict(np.c_[qx, qy], return_std=True)
    return mu + h.prior_mean, np.maximum(sd * sd - h.sn2, 0.0)


def sets(mu, sd, beta, f_min):
    c = beta * sd
    lo = mu - c
    hi = mu + c
    return lo, hi, (lo > f_min).astype(np.uint8)


def gp_case(wl: T.Workload):
    mu, var = gp_numpy(wl.x, wl.y, wl.obs, wl.qx, wl.qy, wl.hyper)
    smu, svar = gp_sklearn(wl.x, wl.y, wl.obs, wl.qx, wl.qy, wl.hyper)
    assert np.abs(mu - smu).max() < 1e-8 * max(1.0, np.abs(mu).max()), "numpy vs sklearn mean"
    assert np.abs(var - svar).max() < 1e-8, "numpy vs sklearn variance"
    sd = np.sqrt(var)
    lo, hi, s = sets(mu, sd, wl.beta, wl.f_min)
    h = wl.hyper
    return dict(x=wl.x, y=wl.y, obs=wl.obs, qx=wl.qx, qy=wl.qy, mu=mu, var=var, sd=sd,
                lo=lo, hi=hi, safe=s, width=wl.width, height=wl.height,
                hyper=np.array([h.length_scale, h.sigma_f, h.noise_level, h.prior_mean]),
                beta=wl.beta, f_min=wl.f_min)


def lpsc_case():
    """lpsc.yaml box [0,1] x [0,2.5] (config/lpsc.yaml:32-33), N=64."""
    h = T.Hyper()
    u = T.uniform(11, 128)
    x = u[0::2] * 1.0
    y = u[1::2] * 2.5
    obs = T.smooth_field(x, y, 2.5, h.length_scale, 11) + np.sqrt(h.sn2) * T.normal(12, 64)
    gx = np.linspace(0.0, 1.0, 12)
    gy = np.linspace(0.0, 2.5, 30)
    QY, QX = np.meshgrid(gy, gx, indexing="ij")
    return T.Workload("lpsc", x, y, obs, QX.reshape(-1), QY.reshape(-1), 12, 30, h,
                      float(np.percentile(obs, 40.0)))


# --------------------------------------------------------------- contours
def _mask(h, w, ones):
    m = np.zeros((h, w), np.uint8)
    for (x, y) in ones:
        m[y, x] = 255
    return m


def contour_cases():
    cases = []
    m = np.zeros((5, 5), np.uint8); m[1:4, 1:4] = 255
    cases.append(("square3", m, [[[1, 1], [1, 2], [1, 3], [2, 3], [3, 3], [3, 2], [3, 1], [2, 1]]]))
    m = np.zeros((3, 3), np.uint8); m[1, 1] = 255
    cases.append(("single_pixel", m, [[[1, 1]]]))
    m = np.zeros((5, 7), np.uint8); m[2, 1:6] = 255
    cases.append(("hline_duplicates", m,
                  [[[1, 2], [2, 2], [3, 2], [4, 2], [5, 2], [4, 2], [3, 2], [2, 2]]]))
    m = np.full((3, 4), 255, np.uint8)
    cases.append(("edge_touching", m,
                  [[[0, 0], [0, 1], [0, 2], [1, 2], [2, 2], [3, 2], [3, 1], [3, 0], [2, 0], [1, 0]]]))
    m = np.zeros((7, 7), np.uint8); m[1:6, 1:6] = 255; m[2:5, 2:5] = 0; m[3, 3] = 255
    ring = [[1, 1], [1, 2], [1, 3], [1, 4], [1, 5], [2, 5], [3, 5], [4, 5], [5, 5],
            [5, 4], [5, 3], [5, 2], [5, 1], [4, 1], [3, 1], [2, 1]]
    cases.append(("lake_with_island", m, [ring]))
    m = np.zeros((6, 6), np.uint8); m[0:2, 4:6] = 255; m[3:5, 0:2] = 255
    cases.append(("two_blobs_reverse_order", m,
                  [[[0, 3], [0, 4], [1, 4], [1, 3]], [[4, 0], [4, 1], [5, 1], [5, 0]]]))
    m = np.zeros((4, 4), np.uint8)
    cases.append(("empty", m, []))
    return cases


def main():
    out = {}
    cases = {
        "lpsc": lpsc_case(),
        "syn256": T.synthetic(256, 32, seed=3),
        "syn1024": T.synthetic(1024, 48, 40, seed=4),
    }
    for k, wl in cases.items():
        for f, v in gp_case(wl).items():
            out[f"{k}__{f}"] = np.asarray(v)
    np.savez_compressed(os.path.join(HERE, "gp_cases.npz"), **out)

    terrain = T.make_terrain_csv()
    T.write_terrain_csv(os.path.join(HERE, "terrain.csv"), terrain)
    terrain = T.load_terrain_csv(os.path.join(HERE, "terrain.csv"))
    c1 = T.c1_workload(terrain)
    c1d = gp_case(c1)
    np.savez_compressed(os.path.join(HERE, "c1.npz"), **{k: np.asarray(v) for k, v in c1d.items()})

    js = [{"name": n, "h": int(m.shape[0]), "w": int(m.shape[1]),
           "mask": m.astype(int).tolist(), "contours": c} for (n, m, c) in contour_cases()]
    with open(os.path.join(HERE, "contours.json"), "w") as f:
        json.dump(js, f, indent=0)
    print("wrote gp_cases.npz, c1.npz, terrain.csv, contours.json")


if __name__ == "__main__":
    main()
