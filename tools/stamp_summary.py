"""Per-workgroup timing of the persistent predictive sweep from the
diagnostic build (-DSBO_STAMPS, libsbo_stamps.so: s_memtime at entry, after
the prologue and at the end, HW_ID/XCC_ID, items and tiles per workgroup,
written to a device array -- no printf).  Runs two ticks and prints the
per-tile sweep cost and the tail imbalance across workgroups.

  SBO_LIB=$PWD/safe_bayesian_optimization_amd/lib/libsbo_stamps.so python tools/stamp_summary.py --config C4"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="C4")
    p.add_argument("--opt", nargs="*", default=[])
    a = p.parse_args()
    import torch
    from safe_bayesian_optimization_amd import TerrainMapper, synthetic
    from safe_bayesian_optimization_amd import _native as N
    from safe_bayesian_optimization_amd.terrain import CONFIGS
    n, gw, gh = CONFIGS[a.config]
    wl = synthetic(n, gw, gh, seed=0)
    dev = torch.device("cuda:0")
    t = lambda v: torch.as_tensor(np.ascontiguousarray(v, np.float32), device=dev)  # noqa: E731
    gm = TerrainMapper(0, wl.hyper)
    for kv in a.opt:
        k, v = kv.split("=")
        gm.set_option(getattr(N, k), int(v))
    gm.fit(t(wl.x), t(wl.y), t(wl.obs))
    qx, qy = t(wl.qx), t(wl.qy)
    m = qx.numel()
    outs = dict(mu=torch.empty(m, device=dev), sd=torch.empty(m, device=dev))
    for _ in range(2):
        gm.tick(qx, qy, wl.beta, wl.f_min, outputs=outs)
    torch.cuda.synchronize()
    wgs = 4096
    buf = np.zeros(wgs * 6, np.uint64)
    rc = N.lib().sbo_debug_stamps(ctypes.c_void_p(buf.ctypes.data), ctypes.c_int64(wgs))
    assert rc == 0, rc
    s = buf.reshape(wgs, 6).astype(np.int64)
    s = s[s[:, 3] > 0]
    st0, st1, st3 = s[:, 0], s[:, 1], s[:, 3]
    items = s[:, 5] >> 32
    tiles = s[:, 5] & 0xFFFFFFFF
    dur = st3 - st0
    pro = st1 - st0
    print(f"{len(s)} persistent workgroups; tiles per WG mean {tiles.mean():.0f} (min {tiles.min()}, max {tiles.max()}), "
          f"items per WG mean {items.mean():.0f}")
    print(f"WG duration (cycles): mean {dur.mean():.4g}  min {dur.min():.4g}  max {dur.max():.4g}  "
          f"-> tail imbalance max/mean {dur.max() / dur.mean():.4f}")
    print(f"prologue median {np.median(pro):.0f} cycles; sweep cycles per tile {((dur - pro).sum() / tiles.sum()):.0f} "
          f"(ideal MFMA 16384: {16384 / ((dur - pro).sum() / tiles.sum()) * 100:.1f} %)")
    xcc = s[:, 4] >> 32
    for x in np.unique(xcc):
        sel = xcc == x
        print(f"  XCC {x}: {sel.sum()} WGs, duration mean {dur[sel].mean():.4g} max {dur[sel].max():.4g}, "
              f"cycles/tile {((dur - pro)[sel].sum() / tiles[sel].sum()):.0f}")
    bid = np.nonzero(buf.reshape(wgs, 6)[:, 3] > 0)[0]
    rng = (bid % 8) * (len(bid) // 8) + bid // 8
    o = np.argsort(rng)
    d = (dur / tiles)[o]
    print("  cycles/tile by range (16 groups, range order): " + " ".join(f"{v:.0f}" for v in d.reshape(16, -1).mean(1)))
    wb = np.zeros(64 * 8 * 5, np.uint64)
    if N.lib().sbo_debug_wave_stamps(ctypes.c_void_p(wb.ctypes.data)) == 0:
        w = wb.reshape(64, 8, 5).astype(np.float64)
        w = w[w[:, 0, 4] > 0]
        steps = w[:, :, 4:5]
        per = (w[:, :, :4] / steps).mean(0)   # [wave][segment] cycles per step
        print("  per step, by wave (cycles): stage-issue | tile MFMA+outer | epilogue+vmcnt | barrier wait")
        for wv in range(8):
            print(f"    wave {wv}: " + " | ".join(f"{v:7.0f}" for v in per[wv]) + f"   total {per[wv].sum():.0f}")
    print(f"cycles per item beyond its tiles' share: "
          f"{((dur - pro).sum() - tiles.sum() * np.median((dur - pro) / tiles)) / items.sum():.0f}")


if __name__ == "__main__":
    main()
