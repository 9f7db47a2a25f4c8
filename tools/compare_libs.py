"""Bitwise A/B of two libsbo builds on the same ticks (GPU): each library runs
in its own process (SBO_LIB), writes the fit's tile bounds, mu/sd/lo/hi/S and the key of a few
workloads, and the outputs are compared element by element.

  python tools/compare_libs.py LIB_A LIB_B [--configs C4 C2 box]"""
import argparse
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys, numpy as np, torch
sys.path.insert(0, {root!r})
from safe_bayesian_optimization_amd import TerrainMapper, synthetic
from safe_bayesian_optimization_amd import _native as N
from safe_bayesian_optimization_amd.terrain import CONFIGS, synthetic_box
out = {{}}
dev = torch.device("cuda:0")
for name in {configs!r}:
    if name == "box":
        wl = synthetic_box(4096, 256, 256, seed=1)
    else:
        n, gw, gh = CONFIGS[name]
        wl = synthetic(n, gw, gh, seed=0)
    t = lambda a: torch.tensor(np.ascontiguousarray(a, np.float32), device=dev)
    gm = TerrainMapper(0, wl.hyper)
    gm.fit(t(wl.x), t(wl.y), t(wl.obs))
    nI = (gm.n + 255) // 256
    b = np.empty(8 * sum(4 * (I + 1) for I in range(nI)), np.float32)   # the plan's tile bounds
    gm.ctx.check(N.lib().sbo_get_tile_bounds(gm.ctx.handle, b.ctypes.data, b.size))
    out[name + "_tile_bounds"] = b
    m = wl.qx.size
    o = dict(mu=torch.empty(m, device=dev), sd=torch.empty(m, device=dev),
             lo=torch.empty(m, dtype=torch.float64, device=dev), hi=torch.empty(m, dtype=torch.float64, device=dev),
             safe=torch.empty(m, dtype=torch.uint8, device=dev))
    k = gm.tick(t(wl.qx), t(wl.qy), wl.beta, wl.f_min, outputs=o).clone()
    torch.cuda.synchronize()
    for kk, v in o.items():
        out[name + "_" + kk] = v.cpu().numpy()
    out[name + "_key"] = k.cpu().numpy()
    gm.close()
np.savez({path!r}, **out)
print("ok", N.LIB_PATH)
'''


def run(lib, configs, path):
    env = dict(os.environ, SBO_LIB=os.path.abspath(lib))
    r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, configs=configs, path=path)], env=env,
                       capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise SystemExit(f"{lib}: {r.stderr[-3000:]}")
    print(r.stdout.strip().splitlines()[-1])
    return dict(np.load(path))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("lib_a")
    p.add_argument("lib_b")
    p.add_argument("--configs", nargs="+", default=["C4", "C2", "box"])
    a = p.parse_args()
    A = run(a.lib_a, a.configs, os.environ.get("CMP_OUT", "/tmp") + "/cmp_a.npz")
    B = run(a.lib_b, a.configs, os.environ.get("CMP_OUT", "/tmp") + "/cmp_b.npz")
    same = True
    for k in sorted(A):
        eq = np.array_equal(A[k], B[k])
        d = "" if eq else f" max|d| {np.abs(A[k].astype(np.float64) - B[k].astype(np.float64)).max():.3e}, " \
                          f"{np.count_nonzero(A[k] != B[k])} of {A[k].size} differ"
        print(f"{k:14s} {'bitwise equal' if eq else 'DIFFERENT'}{d}")
        same &= eq
    print("ALL BITWISE EQUAL" if same else "OUTPUTS DIFFER")
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
