"""MI355X-native GP posterior + acquisition hot path of safe_bayesian_optimization.

Layout:
  csrc/       HIP kernels for gfx950, host orchestration (rocSOLVER) and the
              C ABI of libsbo.so (declared in include/sbo.h)
  _native.py  ctypes binding (no fallback: missing library -> error)
  gp.py       TerrainMapper -- the GP mapper behind get_terrain_map_with_uncertainty
  node.py     OptimizerCore -- mirror of OptimizerNode's ComputeSets /
              FindSafetyContourIndices / GetNextSubgoal
  dist.py     M-row sharding + the cross-rank argmax key reduction
  terrain.py  synthetic workloads (SplitMix64) and the terrain.csv stand-in
"""
from .terrain import Hyper, Workload, synthetic  # noqa: F401

__all__ = ["Hyper", "Workload", "synthetic", "TerrainMapper", "OptimizerCore", "Context"]


def __getattr__(name):
    if name in ("TerrainMapper", "Context", "TerrainMapResponse"):
        from . import gp
        return getattr(gp, name)
    if name == "OptimizerCore":
        from .node import OptimizerCore
        return OptimizerCore
    raise AttributeError(name)
