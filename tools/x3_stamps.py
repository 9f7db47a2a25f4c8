"""Phase shares of the split sweep from its stamp build (variant 39; diagnostic, GPU).

  python tools/x3_stamps.py --config C4
Prints the share of wave-cycles per phase and the body cycles per half-step
by precision level.  Read shares, not lengths: the stamps' waits forbid some
overlap the real kernel has."""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="C4")
    p.add_argument("--variant", type=int, default=39)
    p.add_argument("--opt", nargs="*", default=[], help="NAME=VAL sbo options, e.g. SBO_OPT_TILE_SKIP=0")
    p.add_argument("--save", default="", help="save the per-workgroup loop cycles (.npy)")
    p.add_argument("--box", action="store_true", help="the config's N and grid on the lpsc.yaml box")
    a = p.parse_args()
    import torch
    from safe_bayesian_optimization_amd import TerrainMapper, synthetic
    from safe_bayesian_optimization_amd import _native as N
    from safe_bayesian_optimization_amd.terrain import CONFIGS, synthetic_box
    n, gw, gh = CONFIGS[a.config]
    wl = synthetic_box(n, gw, gh, seed=0) if a.box else synthetic(n, gw, gh, seed=0)
    dev = torch.device("cuda:0")
    t = lambda v: torch.as_tensor(np.ascontiguousarray(v, np.float32), device=dev)  # noqa: E731
    gm = TerrainMapper(0, wl.hyper)
    for kv in a.opt:
        k, v = kv.split("=")
        gm.set_option(getattr(N, k), int(v))
    gm.fit(t(wl.x), t(wl.y), t(wl.obs))
    qx, qy = t(wl.qx), t(wl.qy)
    lib = N.lib()
    nwg = 1024
    buf = (ctypes.c_double * (108 + nwg))()
    for v in (3, a.variant):
        gm.set_option(N.SBO_OPT_KERNEL_VARIANT, v)
        gm.tick(qx, qy, wl.beta, wl.f_min)
    lib.sbo_debug_x3_stamps(gm.ctx.handle, buf, 108 + nwg)  # reset
    gm.tick(qx, qy, wl.beta, wl.f_min)
    lib.sbo_debug_x3_stamps(gm.ctx.handle, buf, 108 + nwg)
    c = list(buf)
    tot = c[5]
    names = ["step top (flush, stage)", "half-step body", "item end", "vmcnt wait", "barrier"]
    for i, nm in enumerate(names):
        print(f"{nm:26s} {100 * c[i] / tot:6.2f} %")
    hs = c[9] + c[10] + c[11]
    print(f"half-steps {hs:.0f}, wave-cycles per half-step {tot / max(hs, 1):.0f}")
    for lv, nm in enumerate(("six", "three", "one")):
        if c[9 + lv]:
            print(f"body at {nm:5s} product(s): {c[6 + lv] / c[9 + lv]:7.0f} cycles per half-step ({c[9 + lv]:.0f})")
    print("per wave index: cycles per half-step in step top / body / item end / vmcnt / barrier")
    for w in range(8):
        cw = c[12 + 12 * w: 24 + 12 * w]
        hw = max(cw[9] + cw[10] + cw[11], 1)
        print(f"  wave {w}: " + " / ".join(f"{cw[i] / hw:6.0f}" for i in range(5)))
    wg = np.array(c[108:108 + nwg])
    wg = wg[:np.count_nonzero(wg)]
    if a.save:
        np.save(a.save, wg)
    if wg.size % 8 == 0 and wg.size:
        x = wg.reshape(-1, 8)  # workgroup b runs on XCD b % 8
        print("per XCD mean/mean: " + " ".join(f"{v:.3f}" for v in x.mean(0) / wg.mean()) +
              "  | within-XCD max/XCD-mean: " + " ".join(f"{v:.3f}" for v in x.max(0) / x.mean(0)))
    if wg.size:
        print(f"workgroups {wg.size}: loop cycles mean {wg.mean():.4g}, max/mean {wg.max() / wg.mean():.3f}, "
              f"min/mean {wg.min() / wg.mean():.3f}, p90/mean {np.percentile(wg, 90) / wg.mean():.3f}")


if __name__ == "__main__":
    main()
