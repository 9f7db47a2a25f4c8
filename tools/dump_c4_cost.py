"""Dump the C4 tick plan's per-query sweep cost (sbo_query_cost: the k-tiles
each query's 128-query block multiplies, under the current build's plan) as
the fixture tests/golden/c4_query_cost.npz -- the cost vector the world-2
gloo test (tests/test_dist.py) cuts with dist.cost_balanced_range, so the
multi-rank path is rehearsed on the real plan at C4 size without a GPU.
GPU tool:  python tools/dump_c4_cost.py [out.npz]   (on the GPU box: a path under
gpurun_out/, then copy it to tests/golden/)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from safe_bayesian_optimization_amd import TerrainMapper, synthetic  # noqa: E402
from safe_bayesian_optimization_amd.terrain import CONFIGS  # noqa: E402


def main():
    n, gw, gh = CONFIGS["C4"]
    wl = synthetic(n, gw, gh, seed=0, name="C4")     # bench.py's C4 workload
    gm = TerrainMapper(0, wl.hyper)
    gm.fit(wl.x, wl.y, wl.obs)
    cost = np.asarray(gm.query_cost(np.float32(wl.qx), np.float32(wl.qy)), np.float32)
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "tests", "golden", "c4_query_cost.npz")
    np.savez_compressed(out, cost=cost, n=n, grid=np.array([gw, gh]))
    print(f"{out}: {cost.size} queries, cost {cost.min():.0f}..{cost.max():.0f}, mean {cost.mean():.1f}, "
          f"{os.path.getsize(out)} bytes")


if __name__ == "__main__":
    main()
