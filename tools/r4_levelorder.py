"""Tiles grouped by precision level inside each item (diagnostic build,
SBO_LEVEL_ORDER=1) against ascending k (0) at C4: sweep ms per tick and the
variance / mean difference between the two orders over the whole grid.
    SBO_LIB=.../libsbo_diag.so python tools/r4_levelorder.py"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import ctypes, json, sys, numpy as np, torch
sys.path.insert(0, {root!r})
from safe_bayesian_optimization_amd import TerrainMapper, synthetic
from safe_bayesian_optimization_amd import _native as N
wl = synthetic(16384, 1000, 1000, seed=0)
dev = torch.device("cuda:0")
t = lambda a: torch.tensor(np.ascontiguousarray(a, np.float32), device=dev)
gm = TerrainMapper(0, wl.hyper)
gm.set_option(N.SBO_OPT_PRECISION, 0)
gm.fit(t(wl.x), t(wl.y), t(wl.obs))
qx, qy = t(wl.qx), t(wl.qy)
lib = N.lib()
mu, sd = gm.predict(qx, qy)
lib.sbo_profile(gm.ctx.handle, 1)
for _ in range(20):
    mu, sd = gm.predict(qx, qy)
torch.cuda.synchronize()
pm, pl, fm, fl = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_int64()
lib.sbo_profile_read(gm.ctx.handle, ctypes.byref(pm), ctypes.byref(pl), ctypes.byref(fm), ctypes.byref(fl))
np.save({out!r}, np.stack([mu.cpu().numpy(), sd.cpu().numpy()]))
print(json.dumps(dict(sweep_ms=pm.value / max(pl.value, 1))), flush=True)
"""


def main():
    import numpy as np
    res = {}
    for lv in ("0", "1", "0", "1"):
        out = f"/tmp/lvorder_{lv}.npy"
        r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, out=out)],
                           env=dict(os.environ, SBO_LEVEL_ORDER=lv), capture_output=True, text=True, timeout=300)
        line = [x for x in r.stdout.splitlines() if x.startswith("{")]
        if r.returncode != 0 or not line:
            print(r.stdout[-2000:], r.stderr[-2000:])
            sys.exit(1)
        ms = json.loads(line[-1])["sweep_ms"]
        res.setdefault(lv, []).append(ms)
        print(f"SBO_LEVEL_ORDER={lv}: sweep {ms:.3f} ms", flush=True)
    a, b = np.load("/tmp/lvorder_0.npy").astype(np.float64), np.load("/tmp/lvorder_1.npy").astype(np.float64)
    dv = np.abs(b[1] ** 2 - a[1] ** 2).max() / (a[1] ** 2).max()
    dm = np.abs(b[0] - a[0]).max() / np.abs(a[0]).max()
    print(json.dumps({"ascending_ms": res["0"], "by_level_ms": res["1"], "var_diff": dv, "mu_diff": dm}))


if __name__ == "__main__":
    main()
