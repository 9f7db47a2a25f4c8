"""Per-workgroup phase timing of the predictive kernel from the diagnostic
build (-DSBO_STAMPS, libsbo_stamps.so: s_memtime at entry, after the tile
list, after the first stage, after the sweep, plus HW_ID/XCC_ID, row block
and tile count per workgroup, written to a device array -- no printf).
Runs one C4 tick and prints where the workgroup time goes, and the idle gap
between consecutive workgroups on the same CU (dispatch cost).

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
    nq = (m + 127) // 128
    nI = -(-n // 256)
    wgs = min(nq * nI, 1 << 20)
    buf = np.zeros(wgs * 6, np.uint64)
    rc = N.lib().sbo_debug_stamps(ctypes.c_void_p(buf.ctypes.data), ctypes.c_int64(wgs))
    assert rc == 0, rc
    s = buf.reshape(wgs, 6).astype(np.int64)
    st0, st1, st2, st3 = s[:, 0], s[:, 1], s[:, 2], s[:, 3]
    hw, meta = s[:, 4], s[:, 5]
    tiles = meta & 0xFFFFFFFF
    I = meta >> 32
    busy = tiles > 0
    lst, first, sweep = st1 - st0, st2 - st1, st3 - st2
    cu = ((hw >> 32) << 16) | (((hw >> 8) & 0xF) << 8) | (((hw >> 13) & 0x1) << 4) | ((hw >> 12) & 0x1)
    # cu key: xcc, cu_id (bits 11:8), sh_id (12), se_id (15:13)
    cu = ((hw >> 32) << 12) | (((hw >> 13) & 0x7) << 6) | (((hw >> 12) & 0x1) << 5) | ((hw >> 8) & 0xF)
    span = st3.max() - st0.min()
    print(f"{wgs} workgroups, {np.mean(~busy) * 100:.1f}% empty, {tiles.sum()} tiles, {len(np.unique(cu))} CUs seen")
    print(f"kernel span {span:.3e} cycles; busy-WG mean tiles {tiles[busy].mean():.2f}")
    tot = (st3 - st0).sum()
    print(f"share of WG-resident cycles: list {lst.sum() / tot * 100:.1f}%  first stage {first[busy].sum() / tot * 100:.1f}%  "
          f"sweep {sweep[busy].sum() / tot * 100:.1f}%  (empty WGs {(st3 - st0)[~busy].sum() / tot * 100:.1f}%)")
    print(f"sweep cycles per tile: {sweep[busy].sum() / tiles[busy].sum():.0f} (median per WG "
          f"{np.median(sweep[busy] / tiles[busy]):.0f});  list median busy {np.median(lst[busy]):.0f} empty "
          f"{np.median(lst[~busy]):.0f};  first stage median {np.median(first[busy]):.0f}")
    # per-CU timelines: idle gap between one WG's end and the next WG's start
    order = np.lexsort((st0, cu))
    c, b, e = cu[order], st0[order], st3[order]
    same = c[1:] == c[:-1]
    gaps = (b[1:] - e[:-1])[same]
    per_cu_busy = np.zeros(0)
    print(f"gap between consecutive WGs on a CU: median {np.median(gaps):.0f}, mean {gaps.mean():.0f} cycles; "
          f"total gaps / total span x CUs = {gaps.sum() / (span * len(np.unique(cu))) * 100:.1f}%")
    for lo, hi in ((0, 8), (8, 32), (32, nI - 1), (nI - 1, nI)):
        sel = busy & (I >= lo) & (I < hi)
        if sel.any():
            print(f"  I in [{lo},{hi}): {sel.sum()} busy WGs, mean tiles {tiles[sel].mean():.1f}, sweep/tile "
                  f"{sweep[sel].sum() / tiles[sel].sum():.0f}, first {np.median(first[sel]):.0f}, list {np.median(lst[sel]):.0f}")


if __name__ == "__main__":
    main()
