"""Level rank keys (SkipPlan::lvl_key) re-calibration A/B at C4 (diagnostic
build, SBO_LVL_KEY): per key pair, the sweep's ms per tick (sbo_profile), the
tiles per level and the variance error against the dense sweep on a sample.
GPU diagnostic:  SBO_LIB=.../libsbo_diag.so python tools/r4_lvlkey.py"""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import ctypes, json, os, sys, numpy as np, torch
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
for _ in range(10):
    mu, sd = gm.predict(qx, qy)
torch.cuda.synchronize()
pm, pl, fm, fl = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_int64()
lib.sbo_profile_read(gm.ctx.handle, ctypes.byref(pm), ctypes.byref(pl), ctypes.byref(fm), ctypes.byref(fl))
mf = ctypes.c_double(); lv = (ctypes.c_int64 * 3)()
lib.sbo_profile_mfma(gm.ctx.handle, ctypes.byref(mf), lv)
np.save({out!r}, sd.cpu().numpy())
print(json.dumps(dict(key=os.environ.get("SBO_LVL_KEY", "default"), sweep_ms=pm.value / max(pl.value, 1),
                      levels=[v / max(pl.value, 1) for v in lv])), flush=True)
"""


def main():
    keys = sys.argv[1:] or ["0.80,1.72", "0.40,1.54", "0.0,1.2", "1.2,2.0", "0.6,1.3"]
    ref = None
    for k in keys:
        out = f"/tmp/lvlkey_{k.replace(',', '_')}.npy"
        env = dict(os.environ, SBO_LVL_KEY=k)
        r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, out=out)], env=env, capture_output=True,
                           text=True, timeout=300)
        line = [x for x in r.stdout.splitlines() if x.startswith("{")]
        if r.returncode != 0 or not line:
            print(r.stdout[-2000:], r.stderr[-2000:])
            sys.exit(1)
        import numpy as np
        res = json.loads(line[-1])
        sd = np.load(out).astype(np.float64)
        if ref is None:
            ref = sd
        res["var_vs_first_key"] = float(np.abs(sd ** 2 - ref ** 2).max() / (ref ** 2).max())
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
