"""The multi-GPU path's collectives on RCCL under a
one-rank nccl process group on cuda:0: every collective bench.py runs at
N > 1 -- the 16-byte key all-gather, the cost-cut broadcast, the fitted
state broadcast + import, the full-grid gather for the node's frontier, the
max-over-ranks timing reduction -- executed by RCCL on device tensors and
checked against the values the N = 1 path computes without a collective.
(The pool's boxes have one GPU, so this is where RCCL first runs before the
driver's 8-GPU node.)"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from safe_bayesian_optimization_amd import TerrainMapper, synthetic  # noqa: E402
from safe_bayesian_optimization_amd.dist import (allreduce_key, combine_keys, cost_balanced_range,  # noqa: E402
                                                gather_rows, key_tensor_to_pairs, rank_cuts, sharded_subgoal)


@pytest.fixture(scope="module")
def pg():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.distributed as dist
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    yield dev
    dist.destroy_process_group()


def _outs(m, dev):
    return dict(mu=torch.empty(m, dtype=torch.float32, device=dev), sd=torch.empty(m, dtype=torch.float32, device=dev),
                lo=torch.empty(m, dtype=torch.float64, device=dev), hi=torch.empty(m, dtype=torch.float64, device=dev),
                safe=torch.empty(m, dtype=torch.uint8, device=dev))


def test_rccl_collectives_of_the_sharded_tick(pg):
    import torch.distributed as dist
    dev = pg
    wl = synthetic(3000, 160, 120, seed=71)
    gm = TerrainMapper(0, wl.hyper)
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a, np.float32), device=dev)  # noqa: E731
    gm.fit(t(wl.x), t(wl.y), t(wl.obs))
    qx, qy = t(wl.qx), t(wl.qy)
    m = qx.numel()
    # cost cut broadcast (nccl, device int64): one rank owns the whole grid
    lo, hi = cost_balanced_range(gm, qx, qy, 0, 1)
    assert (lo, hi) == (0, m)
    outs = _outs(m, dev)
    key = gm.tick(qx, qy, wl.beta, wl.f_min, outputs=outs)
    torch.cuda.synchronize()
    want = key_tensor_to_pairs(key)[0]
    # the tick's 16-byte key through RCCL's all-gather
    assert allreduce_key(key) == want == combine_keys([want])
    # the bench's max-over-ranks of its timings (nccl all_reduce MAX, f64)
    v = torch.tensor([1.5, -2.0, 3.25], dtype=torch.float64, device=dev)
    dist.all_reduce(v, op=dist.ReduceOp.MAX)
    assert v.cpu().tolist() == [1.5, -2.0, 3.25]
    # the fitted state: export, broadcast, import into a second context
    blob = gm.export_state()
    size = torch.tensor([blob.numel()], dtype=torch.int64, device=dev)
    dist.broadcast(size, 0)
    got = torch.empty(int(size.item()), dtype=torch.uint8, device=dev)
    got.copy_(blob)
    dist.broadcast(got, 0)
    assert torch.equal(got, blob)
    other = TerrainMapper(0, wl.hyper)
    other.import_state(got)
    o2 = _outs(m, dev)
    k2 = other.tick(qx, qy, wl.beta, wl.f_min, outputs=o2)
    torch.cuda.synchronize()
    assert torch.equal(k2, key)
    for name in outs:
        assert torch.equal(outs[name], o2[name]), name
    # the full-grid exchange for GetNextSubgoal: cuts, gathered rows, subgoal
    cuts = rank_cuts(lo, hi, device=dev)
    assert cuts == [0, m]
    for name in ("lo", "hi", "safe", "mu"):
        assert torch.equal(gather_rows(outs[name], cuts), outs[name]), name
    Dx = torch.as_tensor(wl.qx, dtype=torch.float64, device=dev)
    Dy = torch.as_tensor(wl.qy, dtype=torch.float64, device=dev)
    goal = (float(wl.qx.mean()), float(wl.qy.mean()))

    def fn(Dx_, Dy_, lo_, hi_, s_, w_, h_, gx, gy):
        return gm.ctx.subgoal(Dx_, Dy_, lo_, hi_, s_, w_, h_, gx, gy)

    idx = sharded_subgoal(fn, Dx, Dy, outs["lo"], outs["hi"], outs["safe"], cuts, wl.width, wl.height, goal)
    assert idx == gm.ctx.subgoal(Dx, Dy, outs["lo"], outs["hi"], outs["safe"], wl.width, wl.height, *goal) >= 0
    other.close()
    gm.close()
