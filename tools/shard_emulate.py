"""Emulate the M-sharded multi-GPU sweep on one GPU (diagnostic): fit once,
then time the planning tick of every rank's contiguous row block
(dist.shard_range) in turn.  Prints per-shard tick time and the whole-job
throughput the sharded run would report (M / the slowest shard), i.e. the
strong-scaling efficiency to expect from `bench.py --gpus P` before the
collective and launch skew.

  python tools/shard_emulate.py --config C4 --world 2 4 8 --reps 5"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="C4")
    p.add_argument("--world", type=int, nargs="+", default=[1, 2, 4, 8])
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--balance", type=float, nargs="*", default=[],
                   help="also try work-balanced cuts (dist.query_work_estimate radius in length scales; "
                        "0 = the plan's own cost, sbo_query_cost)")
    a = p.parse_args()
    import torch
    from safe_bayesian_optimization_amd import TerrainMapper, synthetic
    from safe_bayesian_optimization_amd.dist import balanced_shard_range, query_work_estimate, shard_range
    from safe_bayesian_optimization_amd.terrain import CONFIGS
    n, gw, gh = CONFIGS[a.config]
    wl = synthetic(n, gw, gh, seed=0, name=a.config)
    dev = torch.device("cuda:0")
    f32 = lambda v: torch.as_tensor(np.ascontiguousarray(v, np.float32), device=dev)  # noqa: E731
    gm = TerrainMapper(0, wl.hyper)
    gm.ctx.set_stream(torch.cuda.current_stream(dev))
    gm.fit(f32(wl.x), f32(wl.y), f32(wl.obs))
    m_total = wl.qx.size
    base = None
    for rad in [None] + list(a.balance):
        if rad is None:
            wts = None
        elif rad == 0:
            wts = gm.query_cost(f32(wl.qx), f32(wl.qy)).cpu().numpy()
        else:
            wts = query_work_estimate(wl.qx, wl.qy, wl.x, wl.y, wl.hyper.length_scale, rad)
        for P in a.world:
            ms = []
            for r in range(P):
                lo, hi = shard_range(m_total, r, P) if wts is None else balanced_shard_range(wts, r, P)
                qx, qy = f32(wl.qx[lo:hi]), f32(wl.qy[lo:hi])
                m = hi - lo
                outs = dict(mu=torch.empty(m, device=dev), sd=torch.empty(m, device=dev),
                            lo=torch.empty(m, dtype=torch.float64, device=dev),
                            hi=torch.empty(m, dtype=torch.float64, device=dev),
                            safe=torch.empty(m, dtype=torch.uint8, device=dev))
                # the bench's step on this rank: the tick (async, device key)
                # and the device combine of the P gathered 16-byte keys
                # (sbo_keys_reduce; the all-gather itself, P x 16 B over xGMI,
                # is not emulated)
                key = torch.empty(2, dtype=torch.int64, device=dev)
                gathered = torch.zeros(2 * P, dtype=torch.int64, device=dev)
                best = torch.empty(2, dtype=torch.int64, device=dev)

                def step():
                    gm.tick(qx, qy, wl.beta, wl.f_min, outputs=outs, key_out=key, async_=True)
                    gathered[:2].copy_(key)
                    gm.ctx.reduce_keys(gathered, best)
                step()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.reps):
                    step()
                torch.cuda.synchronize()
                ms.append((time.perf_counter() - t0) * 1e3 / a.reps)
            value = m_total / (max(ms) * 1e-3)
            base = base or value
            tag = "equal" if rad is None else ("plan-cost balanced" if rad == 0 else f"balanced r={rad}")
            print(f"{tag} P={P}: shard tick ms min {min(ms):.2f} mean {np.mean(ms):.2f} max {max(ms):.2f}  "
                  f"-> {value / 1e6:.2f}e6 points/s ({value / base:.2f}x of P={a.world[0]})", flush=True)
    gm.close()


if __name__ == "__main__":
    main()
