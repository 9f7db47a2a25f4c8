"""M-row sharding and the cross-rank argmax key reduction (CPU, gloo)."""
import os
import socket
import struct

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O
from safe_bayesian_optimization_amd.dist import (allreduce_key, balanced_cuts, combine_keys, cost_balanced_range,
                                                shard_range)


def test_shard_range_partitions():
    for m in [1, 7, 256, 1000003]:
        for world in [1, 2, 3, 8]:
            spans = [shard_range(m, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == m
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sharded_argmax_equals_global(world):
    rng = np.random.default_rng(world)
    m = 5000
    score = np.round(rng.uniform(0, 10, m), 1)   # many ties across shards
    mask = (rng.uniform(size=m) < 0.6).astype(np.uint8)
    keys = []
    for r in range(world):
        a, b = shard_range(m, r, world)
        i, v = O.argmax(score[a:b], mask[a:b])
        keys.append((v, a + i if i >= 0 else -1))
    assert combine_keys(keys)[1] == O.argmax(score, mask)[0]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, score, mask, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a, b = shard_range(score.size, rank, world)
    i, v = O.argmax(score[a:b], mask[a:b])
    gi = a + i if i >= 0 else -1
    key = torch.tensor([struct.unpack("<q", struct.pack("<d", v))[0], gi], dtype=torch.int64)
    q.put((rank, allreduce_key(key)))
    dist.destroy_process_group()


def test_gloo_world2_key_allgather():
    rng = np.random.default_rng(7)
    m = 4001
    score = np.round(rng.uniform(0, 5, m), 1)
    mask = (rng.uniform(size=m) < 0.5).astype(np.uint8)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, score, mask, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    want = O.argmax(score, mask)
    for _, (s, i) in res:
        assert i == want[0] and s == want[1]


def test_balanced_cuts_partition_and_balance():
    rng = np.random.default_rng(3)
    for m in [1, 100, 5000, 100003]:
        w = rng.gamma(2.0, 1.0, m) * np.linspace(1.0, 4.0, m)   # work rising along the strip order
        for world in [1, 2, 3, 8]:
            c = balanced_cuts(w, world)
            assert c[0] == 0 and c[-1] == m and all(a <= b for a, b in zip(c, c[1:]))
            assert all(x % 128 == 0 for x in c[1:-1])
            if m >= 128 * world * 8:
                share = [w[a:b].sum() for a, b in zip(c, c[1:])]
                # each block within one aligned row block of the ideal share
                assert max(share) - w.sum() / world <= 128 * w.max() + 1e-9


class _FakeMapper:
    def __init__(self, cost):
        self.cost = cost

    def query_cost(self, qx, qy):
        return self.cost


def _cost_worker(rank, world, port, cost, score, mask, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = cost.size
    qx = torch.zeros(m)
    # only rank 0's mapper knows the costs: the cut must come from the broadcast
    gm = _FakeMapper(cost if rank == 0 else np.ones(m, np.float32))
    a, b = cost_balanced_range(gm, qx, qx, rank, world)
    i, v = O.argmax(score[a:b], mask[a:b])
    gi = a + i if i >= 0 else -1
    key = torch.tensor([struct.unpack("<q", struct.pack("<d", v))[0], gi], dtype=torch.int64)
    q.put((rank, (a, b), allreduce_key(key)))
    dist.destroy_process_group()


def test_gloo_world2_cost_balanced_shards():
    rng = np.random.default_rng(11)
    m = 20000
    cost = np.linspace(1.0, 9.0, m).astype(np.float32)       # the second half costs more
    score = np.round(rng.uniform(0, 5, m), 1)
    mask = (rng.uniform(size=m) < 0.5).astype(np.uint8)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cost_worker, args=(r, 2, port, cost, score, mask, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    (_, s0, k0), (_, s1, k1) = res
    assert s0[0] == 0 and s0[1] == s1[0] and s1[1] == m
    assert s0[1] == balanced_cuts(cost, 2)[1] and s0[1] > m // 2   # the cheap half is the longer one
    want = O.argmax(score, mask)
    for s, i in (k0, k1):
        assert i == want[0] and s == want[1]


# ------------------------------------------------ bench.py's own launcher
def _bench(*args, env=None, timeout=240):
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                          "MASTER_PORT")}
    e.update(env or {})
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, env=e, cwd=root)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r.returncode, (json.loads(lines[-1]) if lines else None), r


@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_launches_its_own_ranks(world):
    """`python bench.py --gpus N` with no WORLD_SIZE starts N ranks itself
    (torch.distributed.run on 127.0.0.1); the JSON line reports the world
    size and backend the collective saw; on a C4-sized (10^6) cost vector the
    cut broadcast balances the work, the key all-gather (host combine and the
    device-path reduce hook) gives the global argmax, and the sharded subgoal
    over uneven row blocks equals the single-rank one (gloo, CPU rehearsal of
    the driver's 8-GPU run)."""
    rc, line, r = _bench("--gpus", str(world), "--launch-check", timeout=600)
    assert rc == 0, r.stderr[-2000:]
    assert line["n_gpus"] == world and line["world_size"] == world and line["backend"] == "gloo"
    assert line["config"]["parallelism"] == f"m-shard{world}"
    assert line["argmax_matches_global"] is True
    assert line["cuts"][0] == 0 and line["cuts"][-1] == 10 ** 6 and len(line["cuts"]) == world + 1
    assert all(c % 128 == 0 for c in line["cuts"][1:-1])
    assert line["cost_share_max_over_mean"] < 1.01
    assert line["subgoal"]["index"] == line["subgoal"]["want"] >= 0


def test_bench_rejects_gpus_world_mismatch():
    rc, line, r = _bench("--gpus", "2", "--launch-check", env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert rc != 0 and line is None and "WORLD_SIZE=1" in r.stderr


# ------------------------------------- full-grid exchange for the frontier
def _subgoal_worker(rank, world, port, cuts, Dx, Dy, lo, hi, s, w, h, goal, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from safe_bayesian_optimization_amd import node as ND
    from safe_bayesian_optimization_amd.dist import gather_rows, rank_cuts, sharded_subgoal
    a, b = cuts[rank], cuts[rank + 1]
    got_cuts = rank_cuts(a, b)
    t = lambda v: torch.as_tensor(np.ascontiguousarray(v))  # noqa: E731
    full_lo = gather_rows(t(lo[a:b]), got_cuts).numpy()

    def fn(Dx_, Dy_, lo_, hi_, s_, w_, h_, gx, gy):
        return ND.next_subgoal(Dx_, Dy_, lo_.numpy(), hi_.numpy(), s_.numpy(), w_, h_, gx, gy)

    idx = sharded_subgoal(fn, Dx, Dy, t(lo[a:b]), t(hi[a:b]), t(s[a:b]), got_cuts, w, h, goal)
    q.put((rank, got_cuts, bool(np.array_equal(full_lo, lo)), idx))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_sharded_subgoal_equals_full(world):
    """Row shards of lo / hi / S (uneven, as cost-balanced cuts give) are
    all-gathered into the full grid on every rank, and the subgoal selected
    from them equals the single-rank GetNextSubgoal on the whole grid."""
    from scipy.ndimage import gaussian_filter
    from safe_bayesian_optimization_amd import node as ND
    rng = np.random.default_rng(5 + world)
    w, h = 48, 40
    xs, ys = np.linspace(-2.0, 3.0, w), np.linspace(-1.0, 2.5, h)
    Dx, Dy = np.tile(xs, h), np.repeat(ys, w)
    m = Dx.size
    mu = gaussian_filter(rng.normal(size=(h, w)), 2.0).reshape(-1) * 5
    sd = rng.uniform(0.01, 1.0, size=m)
    lo, hi, s = O.compute_sets(mu, sd, 2.0, float(np.percentile(mu, 30)))
    cuts = [0] + sorted(rng.choice(np.arange(1, m), world - 1, replace=False).tolist()) + [m]
    goal = (2.5, 2.0)
    want = ND.next_subgoal(Dx, Dy, lo, hi, s, w, h, *goal)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_subgoal_worker, args=(r, world, port, cuts, Dx, Dy, lo, hi, s, w, h, goal, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert want >= 0
    for _, got_cuts, lo_ok, idx in res:
        assert got_cuts == cuts and lo_ok and idx == want


# ------------------------------- the real C4 plan's costs
def _c4_plan_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from safe_bayesian_optimization_amd import _native as N
    from safe_bayesian_optimization_amd.dist import allreduce_key_dev, key_tensor_to_pairs
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cost = np.load(os.path.join(root, "tests", "golden", "c4_query_cost.npz"))["cost"]
    m = cost.size
    # only rank 0's "mapper" has the plan; the others must take its cut
    gm = _FakeMapper(cost if rank == 0 else np.ones(m, np.float32))
    qx = torch.zeros(m)
    a, b = cost_balanced_range(gm, qx, qx, rank, world)
    # acquisition scores of the C4 grid, ties across the cut
    rng = np.random.default_rng(2024)
    score = np.round(rng.uniform(0.0, 3.0, m), 3)
    i = int(np.argmax(score[a:b]))
    key = torch.tensor([np.array([score[a + i]]).view(np.int64)[0], a + i], dtype=torch.int64)
    lib = N.lib()

    def lib_reduce(gathered, out):
        """The device reduce hook's contract (Context.reduce_keys) with the
        library's own key combine (sbo_key_combine: CPU-safe), in rank order."""
        best = N.sbo_key(0.0, -1)
        for s, ix in key_tensor_to_pairs(gathered):
            best = lib.sbo_key_combine(best, N.sbo_key(s, ix))
        return torch.tensor([np.array([best.score]).view(np.int64)[0], best.idx], dtype=torch.int64)

    got = key_tensor_to_pairs(allreduce_key_dev(key, lib_reduce))[0]
    q.put((rank, (a, b), got, float(cost[a:b].sum())))
    dist.destroy_process_group()


def test_gloo_world2_c4_plan_costs():
    """World 2 on the C4 tick plan's own per-query costs (tests/golden/
    c4_query_cost.npz, sbo_query_cost of bench.py's C4 fit, dumped by
    tools/dump_c4_cost.py): rank 0 alone holds the costs, both ranks take its
    broadcast cut (128-aligned, the two shares within 0.1 % of each other --
    equal-size halves differ by far more), and the key all-gather through the
    device-path reduce hook with the library's key combine gives the global
    argmax of all 10^6 queries."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cost = np.load(os.path.join(root, "tests", "golden", "c4_query_cost.npz"))["cost"]
    m = cost.size
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c4_plan_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    (_, s0, k0, c0), (_, s1, k1, c1) = res
    assert m == 10 ** 6 and s0[0] == 0 and s0[1] == s1[0] and s1[1] == m and s0[1] % 128 == 0
    assert s0[1] == balanced_cuts(cost, 2)[1]
    assert max(c0, c1) / ((c0 + c1) / 2) < 1.001
    half = [float(cost[:m // 2].sum()), float(cost[m // 2:].sum())]
    assert max(half) / (sum(half) / 2) > 1.05          # equal halves would be off by > 5 %
    score = np.round(np.random.default_rng(2024).uniform(0.0, 3.0, m), 3)
    want = int(np.argmax(score))                        # lowest index among ties
    for s, i in (k0, k1):
        assert i == want and s == score[want]
