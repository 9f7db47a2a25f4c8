"""Round 5: the precise sweep's item order (SBO_OPT_PLAN_BLOCK) on the lpsc
box at N (default 16384) and the bench's 1000 x 1000 grid: for each precise
kernel (OZ_KERNELS, default "3 4") and each block shape (BLOCKS, bi:bq pairs,
"0" = row-block-major), ms per tick (HIP events of the sweep launches,
sbo_profile) and whether mu / sd are bitwise those of the row-block-major
order (they must be: items are independent); REF_ACROSS=1 compares every
kernel with the first one's output instead.  GPU diagnostic, one JSON line.
    python tools/plan_block_ab.py [n]"""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from safe_bayesian_optimization_amd import TerrainMapper  # noqa: E402
from safe_bayesian_optimization_amd import _native as N  # noqa: E402
from safe_bayesian_optimization_amd.terrain import synthetic_box  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    dev = torch.device("cuda:0")
    wl = synthetic_box(n, 1000, 1000, seed=0)
    t = lambda a: torch.tensor(np.ascontiguousarray(a, np.float32), device=dev)  # noqa: E731
    gm = TerrainMapper(0, wl.hyper)
    lib = N.lib()
    kernels = [int(k) for k in os.environ.get("OZ_KERNELS", "3 4").split()]
    blocks = os.environ.get("BLOCKS", "0 4:8 2:16 8:4 1:32").split()
    out = {"n": n}
    across = os.environ.get("REF_ACROSS") == "1"   # compare every kernel with the first one's output
    ref = None
    for kernel in kernels:
        gm.set_option(N.SBO_OPT_PRECISE_KERNEL, kernel)
        gm.fit(t(wl.x), t(wl.y), t(wl.obs))
        qx, qy = t(wl.qx), t(wl.qy)
        if not across:
            ref = None
        for b in blocks:
            v = 0 if b == "0" else (int(b.split(":")[0]) << 8) | int(b.split(":")[1])
            gm.set_option(N.SBO_OPT_PLAN_BLOCK, v)
            mu, sd = gm.predict(qx, qy)     # warm
            lib.sbo_profile(gm.ctx.handle, 1)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            reps = 2
            for _ in range(reps):
                mu, sd = gm.predict(qx, qy)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / reps
            pm, pl = ctypes.c_double(), ctypes.c_int64()
            fm, fl = ctypes.c_double(), ctypes.c_int64()
            lib.sbo_profile_read(gm.ctx.handle, ctypes.byref(pm), ctypes.byref(pl), ctypes.byref(fm), ctypes.byref(fl))
            lib.sbo_profile(gm.ctx.handle, 0)
            if ref is None:
                ref = (mu.clone(), sd.clone())
            same = bool(torch.equal(mu, ref[0]) and torch.equal(sd, ref[1]))
            out[f"k{kernel}_blk{b}"] = {"tick_ms": wall * 1e3, "sweep_ms_per_launch": pm.value / max(pl.value, 1),
                                        "launches": pl.value, "bitwise_equal_to_row_major": same}
            print(f"kernel {kernel} block {b}: tick {wall * 1e3:.1f} ms, bitwise equal {same}", flush=True)
        gm.set_option(N.SBO_OPT_PLAN_BLOCK, 0)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
