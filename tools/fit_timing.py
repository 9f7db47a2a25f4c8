"""Fit (a1 + a2) timing: first fit (allocations, code objects) vs warm refits,
at C3/C4 sizes.   python tools/fit_timing.py [--n 16384] [--reps 3]"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, nargs="+", default=[8192, 16384])
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--chol", type=int, nargs="+", default=[1], help="SBO_OPT_CHOLESKY values to time (1 own, 0 rocSOLVER)")
    p.add_argument("--inv", type=int, nargs="+", default=[1], help="SBO_OPT_INVERSE values to time (1 own recursion, 0 rocSOLVER dtrtri)")
    p.add_argument("--reserve", type=int, nargs="+", default=[0], help="SBO_OPT_CHOL_RESERVE values to time")
    p.add_argument("--overlap", type=int, nargs="+", default=[0], help="SBO_OPT_INV_OVERLAP values to time")
    p.add_argument("--outer", type=int, nargs="+", default=[1024], help="SBO_OPT_CHOL_OUTER values to time")
    p.add_argument("--gemm", type=int, nargs="+", default=[4], help="SBO_OPT_CHOL_GEMM values to time (4: the library default)")
    p.add_argument("--inv-base", type=int, nargs="+", default=[2048], help="SBO_OPT_INV_BASE values to time")
    p.add_argument("--inv-panels", type=int, nargs="+", default=[16], help="SBO_OPT_INV_PANELS values to time")
    p.add_argument("--leaves", type=int, nargs="+", default=[2], help="SBO_OPT_INV_LEAVES values to time")
    p.add_argument("--prec", type=int, nargs="+", default=[-1],
                   help="SBO_OPT_PRECISION values to time (0: no precision probe at the fit)")
    p.add_argument("--oz", type=int, nargs="+", default=[6], help="SBO_OPT_INV_OZ values to time (0 dgemm, 5/6 sliced; 6 the library default)")
    p.add_argument("--diag", type=int, nargs="+", default=[1], help="SBO_OPT_CHOL_DIAG values to time")
    p.add_argument("--check", type=int, nargs="+", default=[1], help="SBO_OPT_INV_CHECK values to time (0: no guard)")
    p.add_argument("--probe", type=str, nargs="+", default=["32:512"],
                   help="SBO_OPT_PROBE_SIZE values to time, as lattice side:training points")
    p.add_argument("--box", action="store_true", help="the lpsc stress box instead of the C3/C4 synthetic layout")
    a = p.parse_args()
    import torch
    from safe_bayesian_optimization_amd import TerrainMapper, synthetic
    from safe_bayesian_optimization_amd.terrain import synthetic_box
    dev = torch.device("cuda:0")
    from safe_bayesian_optimization_amd import _native as N
    for n, ch, inv, rsv, ov, ou, gg, ib, ip, lv, pr, oz, dg, ck, ps in [
            (n, c, i, r, o, u, g, b, q, v, e, z, d, k, s) for n in a.n for c in a.chol for i in a.inv for r in a.reserve
            for o in a.overlap for u in a.outer for g in a.gemm for b in a.inv_base for q in a.inv_panels
            for v in a.leaves for e in a.prec for z in a.oz for d in a.diag for k in a.check for s in a.probe]:
        wl = synthetic_box(n, 64, 64, seed=0) if a.box else synthetic(n, 64, 64, seed=0)
        t = lambda v: torch.as_tensor(np.ascontiguousarray(v, np.float32), device=dev)  # noqa: E731
        X, Y, O = t(wl.x), t(wl.y), t(wl.obs)
        gm = TerrainMapper(0, wl.hyper)
        gm.set_option(N.SBO_OPT_CHOLESKY, ch)
        gm.set_option(N.SBO_OPT_INVERSE, inv)
        gm.set_option(N.SBO_OPT_CHOL_RESERVE, rsv)
        gm.set_option(N.SBO_OPT_INV_OVERLAP, ov)
        gm.set_option(N.SBO_OPT_CHOL_OUTER, ou)
        gm.set_option(N.SBO_OPT_CHOL_GEMM, gg)
        gm.set_option(N.SBO_OPT_INV_BASE, ib)
        gm.set_option(N.SBO_OPT_INV_PANELS, ip)
        gm.set_option(N.SBO_OPT_INV_LEAVES, lv)
        gm.set_option(N.SBO_OPT_PRECISION, pr)
        gm.set_option(N.SBO_OPT_INV_OZ, oz)
        gm.set_option(N.SBO_OPT_CHOL_DIAG, dg)
        gm.set_option(N.SBO_OPT_INV_CHECK, ck)
        side, train = (int(v) for v in ps.split(":"))
        gm.set_option(N.SBO_OPT_PROBE_SIZE, side << 16 | train)
        ts = []
        for _ in range(a.reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            gm.fit(X, Y, O)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        print(f"N={n} cholesky={ch} inverse={'own recursion' if inv else 'rocSOLVER dtrtri'} reserve={rsv} overlap={ov} outer={ou} gemm={gg} inv_base={ib} inv_panels={ip} leaves={lv} precision={pr} inv_oz={oz} diag={dg} check={ck} probe={ps}{' box' if a.box else ''}: first fit {ts[0]:.1f} ms, warm refits {', '.join(f'{v:.1f}' for v in ts[1:])} ms", flush=True)
        gm.close()


if __name__ == "__main__":
    main()
