"""Headline benchmark: GP posterior + acquisition grid-points/sec at N training points.

One "step" = one planning tick over this rank's shard of the grid (SURVEY.md
3.1 without ROS): the fused predictive sweep (K* generated in registers,
V = sf2 L^-1 K*^T on bf16 MFMA with three-way split operands and f32
accumulation, the mean alongside), ComputeSets in f64, the masked argmax of
the confidence width over the safe set, and the cross-rank key exchange (one
RCCL all-gather of 16-byte keys when N > 1).  Inputs (query coordinates) are
resident in HBM before timing starts; mu/sd/lo/hi/S are written to HBM every
step.  The fit (RBF fill, blocked Cholesky, f64 recursive L^-1, alpha,
operand pack, precision probe) runs once, replicated on every rank, and is
reported separately, with the end-to-end rate M / (fit + tick) beside it.

Default workload = BASELINE.json configs[3] (C4: N=16384, 1000x1000 grid),
the north-star target size, on 1 GPU; with --gpus P the same 10^6-point grid
is split into P contiguous, cost-balanced row blocks (strong scaling).
--config C5 runs the streaming loop instead (configs[4]: 50 iterations, N
1000 -> 8000 by incremental Cholesky appends, 512x512 grid, 1 GPU): a step is
one append + one tick.

At N = 1 the same JSON line also carries two regimes measured in the same
run (``regimes``): the C4 sweep with tile skipping off (executed work = the
dense N^2 M of SURVEY.md 8(d)) and the lpsc.yaml stress box
([0, 1] x [0, 2.5], config/lpsc.yaml:32-33) where almost nothing can be
skipped -- so the algorithmic speed-up (skipping) and the hardware speed-up
(GPU vs the dense CPU path) are reported apart.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2|C3|C4|C5]
  (--gpus N > 1 without WORLD_SIZE launches N ranks itself through
   torch.distributed.run on 127.0.0.1; the driver's own
   python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
   is accepted as is)
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_F32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: dense f32 MFMA peak (spec, 2.4 GHz)
PEAK_BF16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA peak (spec; not the 2:1-sparsity figure)
SPLIT_VARIANTS = (2, 3, 22, 23)  # split-operand (bf16 x3) sweeps: up to six bf16 MFMA products per f32 product
PEAK_HBM_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
METRIC = "GP posterior+acq grid-points/sec at N train pts; 1/2/4/8 GPU"
DATA = "synthetic (SplitMix64 smooth field + N(0,sn2) noise in BASELINE config shapes; terrain.csv is a missing blob)"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="ranks (one per GPU); > 1 without WORLD_SIZE launches them itself")
    p.add_argument("--steps", type=int, default=300,
                   help="timed ticks (default 300: ~7 s at C4, long enough for a 5 s utilisation sampler)")
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default="C4", choices=["C2", "C3", "C4", "C5"])
    p.add_argument("--n", type=int, default=None, help="override N")
    p.add_argument("--grid", type=int, default=None, help="override grid side")
    p.add_argument("--scaling", default="strong", choices=["strong", "weak"])
    p.add_argument("--backend", default="nccl", help="torch.distributed backend for N > 1 (nccl = RCCL)")
    p.add_argument("--force-pg", action="store_true",
                   help="initialise the process group (and run every collective of the N > 1 path: key "
                        "all-gather, cut broadcast, state broadcast + import, full-grid gather) even at one rank "
                        "-- RCCL exercised on a one-GPU box")
    p.add_argument("--sharding", default="cost", choices=["cost", "equal"],
                   help="strong scaling: cost-balanced contiguous row blocks (default) or equal point counts")
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU baseline budget (rank 0, N=1)")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-warmup", action="store_true", help="no sbo_warmup before the first fit (cold first fit)")
    p.add_argument("--cpu-child", default=None, help=argparse.SUPPRESS)
    p.add_argument("--no-outputs", action="store_true", help="skip writing mu/sd/lo/hi/S (argmax only)")
    p.add_argument("--no-regimes", action="store_true",
                   help="N = 1: skip the dense (no tile skipping) and lpsc stress-box measurements")
    p.add_argument("--regime-steps", type=int, default=2, help="timed ticks per regime (after one warmup)")
    p.add_argument("--launch-check", action="store_true",
                   help="CPU rehearsal of the multi-rank path (gloo): launcher, shard cut broadcast, key all-gather")
    p.add_argument("--resort", type=int, default=25,
                   help="C5: SBO_OPT_RESORT, re-sort + refactor once appended points exceed this %% (0: never)")
    p.add_argument("--variant", type=int, default=3,
                   help="predictive kernel (SBO_OPT_KERNEL_VARIANT): 3 split-operand bf16 sweep (default), 0 f32 MFMA")
    return p.parse_args()


class Prof:
    """Kernel timing recorded by libsbo on the launch stream (sbo_profile)."""

    def __init__(self, lib, handle):
        self.lib, self.h = lib, handle

    def reset(self, on=True):
        self.lib.sbo_profile(self.h, 1 if on else 0)

    def read(self):
        pm, pl, fm, fl = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_int64()
        self.lib.sbo_profile_read(self.h, ctypes.byref(pm), ctypes.byref(pl), ctypes.byref(fm), ctypes.byref(fl))
        w, mf = ctypes.c_double(), ctypes.c_double()
        lv = (ctypes.c_int64 * 3)()
        self.lib.sbo_profile_work(self.h, ctypes.byref(w))
        self.lib.sbo_profile_mfma(self.h, ctypes.byref(mf), lv)
        return dict(predict_ms=pm.value, predict_launches=pl.value, fill_ms=fm.value, fill_launches=fl.value,
                    predict_flops=w.value, mfma_flops=mf.value, tiles_by_level=list(lv))


def _free_port():
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def launch(a):
    """--gpus N > 1 without a launcher: start N ranks (one process per GPU)
    through torch.distributed.run on 127.0.0.1 and return its exit code.  No
    GPU call has been made in this process (only the children touch it)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # RCCL on this host needs dmabuf IPC
    return subprocess.call(cmd, env=env)


def main():
    a = parse()
    if a.cpu_child:
        return cpu_child(a.cpu_child, a.cpu_seconds)
    if "WORLD_SIZE" not in os.environ and (a.gpus or 1) > 1:
        return launch(a)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus is not None and a.gpus != world:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}")
    if a.launch_check:
        return run_launch_check(a, world, rank)
    import torch
    import torch.distributed as dist

    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local % max(ndev, 1))
    torch.cuda.set_device(dev)
    pg = world > 1 or a.force_pg
    if pg:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(a.backend)
    a.pg = pg
    try:
        if a.config == "C5":
            line = run_streaming(a, dev, world, rank)
        else:
            line = run_sweep(a, dev, world, rank)
        if rank == 0:
            print(json.dumps(line), flush=True)
    finally:
        if pg:
            dist.barrier()
            dist.destroy_process_group()
    return 0


def dist_info(backend):
    """What the collective actually saw (not what was asked for)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return {"world_size": dist.get_world_size(), "backend": str(dist.get_backend()),
                "collective": "all_gather_into_tensor of 16-byte (f64 score, i64 index) keys, one per tick",
                "process_group": True}
    return {"world_size": 1, "backend": None, "collective": None}


def run_launch_check(a, world, rank):
    """The multi-rank path without a GPU (gloo on CPU tensors), at the sizes the
    driver's 8-GPU run uses: the cost-cut broadcast of a
    C4-sized (10^6-query) cost vector that only rank 0 knows
    (dist.cost_balanced_range), the key all-gather combined both ways -- host
    (allreduce_key) and through the reduce hook the GPU path uses
    (allreduce_key_dev; here a host stand-in for the device reduction) -- and
    the full-grid exchange for the frontier (dist.sharded_subgoal: lo/hi/S
    all-gathered from uneven row blocks, GetNextSubgoal on every rank).  Rank
    0 prints a JSON line with what the ranks saw."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from safe_bayesian_optimization_amd import node as ND
    from safe_bayesian_optimization_amd.dist import (allreduce_key, allreduce_key_dev, balanced_cuts, combine_keys,
                                                     cost_balanced_range, key_tensor_to_pairs, rank_cuts,
                                                     sharded_subgoal)
    from safe_bayesian_optimization_amd.terrain import CONFIGS

    if world > 1:
        dist.init_process_group("gloo")
    _, gw, gh = CONFIGS["C4"]
    m = gw * gh
    rng = np.random.default_rng(123)
    # the C4 tick plan's own per-query costs (tools/dump_c4_cost.py), else a
    # C4-shaped stand-in: more tiles in the middle rows than at the edges
    fx = os.path.join(ROOT, "tests", "golden", "c4_query_cost.npz")
    if os.path.exists(fx):
        cost = np.load(fx)["cost"].astype(np.float32)
        cost_src = "tests/golden/c4_query_cost.npz (sbo_query_cost of the C4 fit)"
    else:
        rows = np.repeat(np.sin(np.linspace(0.1, np.pi - 0.1, gh)), gw)
        cost = (0.5 + rows + 0.3 * rng.uniform(size=m)).astype(np.float32)
        cost_src = "synthetic C4-shaped stand-in"
    assert cost.size == m
    score = np.round(rng.uniform(0.0, 4.0, m), 2)   # ties across shards

    class _Rank0Costs:   # only rank 0's "mapper" knows the costs: the cut must come from the broadcast
        def query_cost(self, qx, qy):
            return cost if rank == 0 else np.ones(m, np.float32)

    q = torch.zeros(m)
    lo, hi = cost_balanced_range(_Rank0Costs(), q, q, rank, world)
    cuts = rank_cuts(lo, hi)
    j = int(np.argmax(score[lo:hi])) if hi > lo else -1
    s = float(score[lo + j]) if j >= 0 else 0.0
    key = torch.tensor([np.array([s]).view(np.int64)[0], lo + j if j >= 0 else -1], dtype=torch.int64)
    want = combine_keys([(float(score.max()), int(np.argmax(score)))])
    best = allreduce_key(key)

    def host_reduce(gathered, out):
        sc, ix = combine_keys(key_tensor_to_pairs(gathered))
        return torch.tensor([np.array([sc]).view(np.int64)[0], ix], dtype=torch.int64)

    best_dev = key_tensor_to_pairs(allreduce_key_dev(key, host_reduce))[0]
    # the frontier exchange on a smaller grid with uneven cuts (random costs)
    w, h = 300, 200
    xs, ys = np.linspace(-3.0, 3.0, w), np.linspace(-2.0, 2.0, h)
    Dx, Dy = np.tile(xs, h), np.repeat(ys, w)
    mu = np.sin(1.3 * Dx) * np.cos(0.9 * Dy) * 3 + 0.2 * Dx
    sd = 0.05 + 0.5 * np.abs(np.sin(0.7 * Dx + Dy))
    glo = mu - 2.0 * sd
    ghi = mu + 2.0 * sd
    gs = (glo > -1.0).astype(np.uint8)
    fcuts = balanced_cuts(np.random.default_rng(7).gamma(1.0, 1.0, w * h), world, align=1)
    a0, a1 = fcuts[rank], fcuts[rank + 1]
    t = lambda v: torch.as_tensor(np.ascontiguousarray(v))  # noqa: E731
    goal = (2.0, 1.5)

    def fn(Dx_, Dy_, lo_, hi_, s_, w_, h_, gx, gy):
        return ND.next_subgoal(Dx_, Dy_, lo_.numpy(), hi_.numpy(), s_.numpy(), w_, h_, gx, gy)

    sub = sharded_subgoal(fn, Dx, Dy, t(glo[a0:a1]), t(ghi[a0:a1]), t(gs[a0:a1]), rank_cuts(a0, a1), w, h, goal)
    sub_want = ND.next_subgoal(Dx, Dy, glo, ghi, gs, w, h, *goal)
    ok = best == want and best_dev == want and sub == sub_want and sub_want >= 0
    flags = torch.tensor([1 if ok else 0], dtype=torch.int64)
    if world > 1:
        dist.all_reduce(flags, op=dist.ReduceOp.MIN)
    info = dist_info(a.backend)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        share = [float(cost[c0:c1].sum()) for c0, c1 in zip(cuts, cuts[1:])]
        print(json.dumps({"metric": METRIC, "value": None, "unit": "grid-points/s", "n_gpus": world,
                          "launch_check": True, "argmax_matches_global": bool(flags[0]), "cuts": cuts,
                          "cost_share_max_over_mean": max(share) / (sum(share) / len(share)),
                          "subgoal": {"index": sub, "want": sub_want, "cuts": fcuts}, "cost_source": cost_src,
                          "config": {"workload": "launch-check (C4-sized costs)", "M": m,
                                     "parallelism": f"m-shard{world}" if world > 1 else "single"}, **info}),
              flush=True)
    return 0 if bool(flags[0]) else 1


def _max_over_ranks(vals, dev, world, backend):
    import torch
    import torch.distributed as dist
    if not dist.is_initialized():
        return vals
    t = torch.tensor(vals, dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.cpu()]


def run_sweep(a, dev, world, rank):
    import torch
    import torch.distributed as dist

    from safe_bayesian_optimization_amd import TerrainMapper, synthetic
    from safe_bayesian_optimization_amd import _native as N
    from safe_bayesian_optimization_amd.dist import (allreduce_key, allreduce_key_dev, cost_balanced_range,
                                                     key_tensor_to_pairs, shard_range)
    from safe_bayesian_optimization_amd.gp import _to_hyper
    from safe_bayesian_optimization_amd.terrain import CONFIGS

    n, gw, gh = CONFIGS[a.config]
    n = a.n or n
    if a.grid:
        gw = gh = a.grid
    wl = synthetic(n, gw, gh, seed=0, name=a.config)
    m_total = wl.qx.size
    m_all = m_total * world if a.scaling == "weak" else m_total

    stream = torch.cuda.current_stream(dev)
    gm = TerrainMapper(dev.index, wl.hyper)
    gm.set_option(N.SBO_OPT_KERNEL_VARIANT, a.variant)
    gm.ctx.set_stream(stream)
    lib = N.lib()
    prof = Prof(lib, gm.ctx.handle)

    f32 = lambda v: torch.as_tensor(np.ascontiguousarray(v, np.float32), device=dev)  # noqa: E731
    X, Y, OBS = f32(wl.x), f32(wl.y), f32(wl.obs)
    key = torch.empty(2, dtype=torch.int64, device=dev)

    # ---- fit (replicated on every rank), timed separately: the first fit in
    # the process and a warm refit (what a map update costs in steady state).
    # The node's startup warm-up (sbo_warmup: every code object a fit and a
    # tick load, the workspaces sized for N and M) runs first and is timed on
    # its own, so the first fit is what the node's first map costs
    # (--no-warmup: the cold first fit, code-object loading included)
    warmup_ms = None
    if not a.no_warmup:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gm.warmup(n, m_total)
        torch.cuda.synchronize()
        warmup_ms = (time.perf_counter() - t0) * 1e3
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gm.fit(X, Y, OBS)
    torch.cuda.synchronize()
    fit_first_ms = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    gm.fit(X, Y, OBS)
    torch.cuda.synchronize()
    fit_ms = (time.perf_counter() - t0) * 1e3
    # the warm refit's inverse accuracy guard (SBO_OPT_INV_CHECK: its measured
    # share of the variance error, whether it fell back to dgemm, device ms on
    # its own stream beside the operand packs)
    inv_chk = gm.inverse_check()
    # SURVEY.md 8(e) alternative: rank 0 fits, the packed predictive state is
    # broadcast (RCCL) and imported elsewhere -- timed beside the replicated fit
    fit_bcast = None
    if a.pg:
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        on_dev = a.backend == "nccl"
        size = torch.zeros(1, dtype=torch.int64, device=dev if on_dev else "cpu")
        if rank == 0:
            gm.fit(X, Y, OBS)
            blob = gm.export_state()
            size[0] = blob.numel()
        dist.broadcast(size, 0)
        if rank != 0:
            blob = torch.empty(int(size.item()), dtype=torch.uint8, device=dev)
        if on_dev:
            dist.broadcast(blob, 0)
        else:
            hb = blob.cpu()
            dist.broadcast(hb, 0)
            blob.copy_(hb)
        if rank != 0 or world == 1:
            # (one rank: import the broadcast blob into a second context and
            # check the sweep is bitwise the fitted one's -- the path a
            # receiving rank takes)
            tgt = gm if rank != 0 else TerrainMapper(dev.index, wl.hyper)
            tgt.import_state(blob)
        torch.cuda.synchronize()
        dist.barrier()
        fit_bcast = {"ms": (time.perf_counter() - t0) * 1e3, "state_bytes": int(size.item()),
                     "how": "rank 0 sbo_fit + sbo_export_state, broadcast, sbo_import_state"}
        if world == 1:
            qs = f32(wl.qx[:65536]), f32(wl.qy[:65536])
            ma, sa = gm.predict(*qs)
            mb, sb = tgt.predict(*qs)
            fit_bcast["import_bitwise_equal"] = bool(torch.equal(ma, mb) and torch.equal(sa, sb))
            tgt.close()
        del blob
    # ---- this rank's contiguous block of grid rows (strong scaling): cut so
    # that every rank sweeps about the same number of k-tiles (rank 0 plans
    # all M queries once, sbo_query_cost, and broadcasts the cuts), or equal
    # point counts with --sharding equal
    if a.scaling == "weak":
        lo, hi = 0, m_total
    elif a.pg and a.sharding == "cost":
        lo, hi = cost_balanced_range(gm, f32(wl.qx), f32(wl.qy), rank, world)
    else:
        lo, hi = shard_range(m_total, rank, world)
    m = hi - lo
    qx, qy = f32(wl.qx[lo:hi]), f32(wl.qy[lo:hi])
    outs = {} if a.no_outputs else dict(
        mu=torch.empty(m, dtype=torch.float32, device=dev), sd=torch.empty(m, dtype=torch.float32, device=dev),
        lo=torch.empty(m, dtype=torch.float64, device=dev), hi=torch.empty(m, dtype=torch.float64, device=dev),
        safe=torch.empty(m, dtype=torch.uint8, device=dev))
    cutoff, row_l1, alpha_l1 = gm.skip_info()
    prec = gm.precision()

    # ---- RBF fill (a1) alone, warm (the fill inside fit also paid the code-object load)
    Kbuf = torch.empty(n * n, dtype=torch.float32, device=dev)
    fill_args = (gm.ctx.handle, ctypes.c_void_p(X.data_ptr()), ctypes.c_void_p(Y.data_ptr()), n,
                 _to_hyper(wl.hyper), ctypes.c_void_p(Kbuf.data_ptr()), N.SBO_DEVICE_PTRS | N.SBO_ASYNC)
    gm.ctx.check(lib.sbo_rbf_fill(*fill_args))
    prof.reset()
    for _ in range(3):
        gm.ctx.check(lib.sbo_rbf_fill(*fill_args))
    pr = prof.read()
    fill_ms = pr["fill_ms"] / max(pr["fill_launches"], 1)
    fill_bytes = 4.0 * n * n + 8.0 * n
    del Kbuf

    best_key = torch.empty(2, dtype=torch.int64, device=dev)

    def step():
        gm.tick(qx, qy, wl.beta, wl.f_min, score=N.SCORE_WIDTH, index_offset=lo, outputs=outs, key_out=key,
                async_=True)
        if a.backend == "nccl" or not a.pg:
            # RCCL all-gather of the 16-byte keys, combined on the device (no
            # per-tick host sync); at one rank without a process group the
            # device combine of the one key
            return allreduce_key_dev(key, gm.ctx.reduce_keys, out=best_key)
        return allreduce_key(key.cpu())     # gloo: host tensors, host combine

    for _ in range(a.warmup):
        step()
    prof.reset()   # time only the K measured launches
    if a.pg:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    best = None
    for _ in range(a.steps):
        best = step()
    torch.cuda.synchronize()
    if not isinstance(best, tuple):
        best = key_tensor_to_pairs(best)[0]
    if a.pg:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    pr = prof.read()
    prof.reset(False)
    pred_ms = pr["predict_ms"] / max(pr["predict_launches"], 1)
    exec_flops_launch = pr["predict_flops"] / max(pr["predict_launches"], 1)
    mfma_flops_launch = pr["mfma_flops"] / max(pr["predict_launches"], 1)
    levels_launch = [x / max(pr["predict_launches"], 1) for x in pr["tiles_by_level"]]
    elapsed, pred_ms_max, fit_ms_max = _max_over_ranks([elapsed, pred_ms, fit_ms], dev, world, a.backend)
    subgoal_sharded = None
    if a.pg and not a.no_outputs and a.scaling == "strong":
        # the node-parity frontier needs the whole grid: lo / hi / S of every
        # rank all-gathered (17 B per point, SURVEY.md 8(e) optional exchange),
        # then GetNextSubgoal on every rank -- timed apart from the tick
        from safe_bayesian_optimization_amd.dist import rank_cuts, sharded_subgoal
        on_dev = a.backend == "nccl"
        Dx = torch.as_tensor(wl.qx, dtype=torch.float64, device=dev)
        Dy = torch.as_tensor(wl.qy, dtype=torch.float64, device=dev)
        goal = (float(wl.qx.mean()), float(wl.qy.mean()))
        cuts = rank_cuts(lo, hi, device=dev if on_dev else "cpu")
        loc = [outs[k] if on_dev else outs[k].cpu() for k in ("lo", "hi", "safe")]

        def fn(Dx_, Dy_, lo_, hi_, s_, w_, h_, gx, gy):
            return gm.ctx.subgoal(Dx_, Dy_, lo_.to(dev), hi_.to(dev), s_.to(dev), w_, h_, gx, gy)

        sg = lambda: sharded_subgoal(fn, Dx, Dy, *loc, cuts, gw, gh, goal)  # noqa: E731
        sg()
        torch.cuda.synchronize()
        dist.barrier()
        t1 = time.perf_counter()
        for _ in range(3):
            sidx = sg()
        torch.cuda.synchronize()
        sub_ms = _max_over_ranks([(time.perf_counter() - t1) * 1e3 / 3], dev, world, a.backend)[0]
        subgoal_sharded = {"index": sidx, "ms": sub_ms, "goal": goal, "gathered_bytes": 17 * m_total,
                           "how": "lo/hi/S all-gathered from the row shards (one all_gather each), then "
                                  "sbo_subgoal on every rank (same index everywhere)"}
    winfo = dist_info(a.backend)
    if rank != 0:
        return None

    ms_per_step = elapsed * 1e3 / a.steps
    value = m_all * a.steps / elapsed
    # Algorithmic work of one launch: the MFMA products that are not dropped --
    # 2*BM*BN*BK per k-tile a workgroup multiplies (counted on the device).
    # k-tiles whose every K* entry is below the error-budgeted cutoff 2^-L are
    # skipped.  The dense figure N^2 flop per grid point
    #  is reported beside it as a throughput equivalent.
    dense_flops_launch = float(n) * float(n) * m
    achieved = exec_flops_launch / (pred_ms * 1e-3) / 1e12
    fill_gbs = fill_bytes / (fill_ms * 1e-3) / 1e9 if fill_ms > 0 else None
    # node-side selection on the tick's device outputs (8(f)1): frontier of S,
    # nearest quarter to the goal, widest interval -- GetNextSubgoal
    subgoal = None
    if world == 1 and not a.no_outputs and subgoal_sharded is None:
        Dx = torch.as_tensor(wl.qx, dtype=torch.float64, device=dev)
        Dy = torch.as_tensor(wl.qy, dtype=torch.float64, device=dev)
        goal = (float(wl.qx.mean()), float(wl.qy.mean()))
        sg = lambda: gm.ctx.subgoal(Dx, Dy, outs["lo"], outs["hi"], outs["safe"], gw, gh, *goal)  # noqa: E731
        sg()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(3):
            sidx = sg()
        sub_ms = (time.perf_counter() - t1) * 1e3 / 3
        subgoal = {"index": sidx, "ms": sub_ms, "goal": goal,
                   "how": "sbo_subgoal: device raster/owner map, host border follow of the w x h image"}
    else:
        subgoal = subgoal_sharded
    cpu = cpu_baseline(gm, wl, a.cpu_seconds) if world == 1 and not a.no_cpu else None
    traffic, traffic_src = pmc_traffic(a.config, n, m_total, m)
    regimes = None
    if world == 1 and not a.no_regimes:
        regimes = {"dense": run_regime_dense(a, gm, prof, step, n, m)}
        regimes["append1"] = run_regime_append1(a, gm, dev, wl, qx, qy, outs, key, fit_ms, ms_per_step)
        regimes["lpsc_stress_box"] = run_regime_stress(a, gm, prof, dev, n, gw, gh)
    if cpu is not None:
        cpu["gpu_over_cpu"] = value / cpu["value"]
        if regimes:
            d = regimes["dense"]
            cpu["gpu_dense_over_cpu"] = d["value"] / cpu["value"]
            best_cpu = max(b["value"] for b in cpu["by_threads"])
            for b in cpu["by_threads"]:
                if b["value"] < cpu["value"]:
                    # more threads ran slower than the headline share (OpenBLAS
                    # caps its own threads; oversubscribed cores): a measurement
                    # of the host, not a baseline -- no ratio is quoted against it
                    b["baseline"] = False
                    continue
                b["gpu_dense_over_cpu"] = d["value"] / b["value"]
                b["gpu_over_cpu"] = value / b["value"]
            cpu["gpu_dense_over_best_cpu"] = d["value"] / best_cpu
            cpu["gpu_default_over_gpu_dense"] = value / d["value"]
            cpu["ratios"] = ("gpu_dense_over_cpu: hardware (the same dense algorithm on both; "
                             "gpu_dense_over_best_cpu against the fastest thread count measured); "
                             "gpu_default_over_gpu_dense: algorithmic (error-budgeted tile skipping and "
                             "precision levels, which a CPU could use too); gpu_over_cpu = their product, "
                             "not a hardware ratio; thread counts slower than the headline share carry "
                             "baseline: false and no ratio")
    return {
        "metric": METRIC, "value": value, "unit": "grid-points/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": a.scaling,
        "vs_baseline": None, "dtype": "f64" if prec[0] else dtype_of(a.variant), "data": DATA,
        "world_size": winfo["world_size"], "backend": winfo["backend"], "collective": winfo["collective"],
        "config": {"workload": a.config, "n_train": n, "grid": [gw, gh], "M": m_total, "M_per_rank": m,
                   "beta": wl.beta, "f_min": round(wl.f_min, 6),
                   "hyper": [wl.hyper.length_scale, wl.hyper.sigma_f, wl.hyper.noise_level],
                   "kstar_cutoff_log2": cutoff, "parallelism": f"m-shard{world}" if world > 1 else "single",
                   "sharding": (a.sharding if world > 1 and a.scaling == "strong" else None),
                   "outputs_written": not a.no_outputs,
                   "precision": {"precise_sweep": prec[0], "probe_fast_sweep_variance_error": prec[1],
                                 "probe_var_min": prec[2], "probe_var_max": prec[3],
                                 "rule": "SBO_OPT_PRECISION -1: the precise sweep when the probe error > 5e-6"}},
        "roofline": dict(predict_roofline(a.variant, exec_flops_launch, pred_ms, mfma_flops_launch, levels_launch,
                                          prec[0], gm.probe_info()["precise_kernel"]),
                         traffic=traffic,
                         traffic_source=traffic_src, avg_launch_ms=pred_ms, max_rank_launch_ms=pred_ms_max,
                         dense_flops_per_launch=dense_flops_launch,
                         executed_fraction_of_dense=exec_flops_launch / dense_flops_launch,
                         dense_equivalent_tflops=dense_flops_launch / (pred_ms * 1e-3) / 1e12),
        "fill_roofline": {"kernel": "rbf_fill_kernel", "bound": "hbm", "achieved": fill_gbs, "peak": PEAK_HBM_GBS,
                          "unit": "GB/s", "frac": (fill_gbs / PEAK_HBM_GBS) if fill_gbs else None,
                          "avg_launch_ms": fill_ms, "algorithmic_bytes": fill_bytes},
        "fit_ms": fit_ms, "fit_first_ms": fit_first_ms, "warmup_ms": warmup_ms,
        "fit_first_how": ("the first sbo_fit after sbo_warmup(N, M) at startup (warmup_ms)" if warmup_ms is not None
                          else "the cold first sbo_fit of the process"),
        "fit_broadcast": fit_bcast,
        "inverse_check": inv_chk,
        "end_to_end": end_to_end(m_all, fit_ms_max, ms_per_step),
        "argmax": {"index": best[1], "score": best[0]},
        "subgoal": subgoal,
        "cpu_baseline": cpu,
        "regimes": regimes,
    }


def end_to_end(m, fit_ms, tick_ms):
    """the tick with a refit in front of it -- the reference's
    trigger requests a new map on every spatial_data_size change
    (node.cpp:552-566), so a fresh map costs the warm fit plus one tick."""
    return {"value": m / ((fit_ms + tick_ms) * 1e-3), "unit": "grid-points/s", "fit_ms": fit_ms,
            "tick_ms": tick_ms, "how": "M / (warm fit + one tick); fit replicated on every rank (max over ranks)"}


def _timed_ticks(prof, step, steps):
    """One warmup tick, then `steps` ticks: (wall s per tick, sweep counters per launch)."""
    import torch
    step()
    prof.reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    pr = prof.read()
    prof.reset(False)
    k = max(pr["predict_launches"], 1)
    return wall, pr["predict_ms"] / k, pr["predict_flops"] / k, pr["mfma_flops"] / k, [x / k for x in pr["tiles_by_level"]]


def _regime_line(a, name, how, m, n, wall, ms, flops, mflops, levels, extra=None, precise=False, precise_kernel=1):
    dense = float(n) * float(n) * m
    r = {"what": how, "value": m / wall, "unit": "grid-points/s", "ms_per_step": wall * 1e3,
         "roofline": dict(predict_roofline(a.variant, flops, ms, mflops, levels, precise, precise_kernel),
                          avg_launch_ms=ms,
                          dense_flops_per_launch=dense, executed_fraction_of_dense=flops / dense,
                          dense_equivalent_tflops=dense / (ms * 1e-3) / 1e12)}
    if extra:
        r.update(extra)
    return r


def run_regime_dense(a, gm, prof, step, n, m):
    """The same C4 tick with tile skipping off (SBO_OPT_TILE_SKIP = 0): every
    k-tile of the lower triangle multiplied at six bf16 products, so executed
    work is the dense N^2 flop per grid point of SURVEY.md 8(d)."""
    from safe_bayesian_optimization_amd import _native as N
    gm.set_option(N.SBO_OPT_TILE_SKIP, 0)
    try:
        res = _timed_ticks(prof, step, a.regime_steps)
    finally:
        gm.set_option(N.SBO_OPT_TILE_SKIP, -1)
    return _regime_line(a, "dense", f"{a.config} tick, SBO_OPT_TILE_SKIP=0 (no skipping, all tiles at six products)",
                        m, n, *res)


def run_regime_append1(a, gm, dev, wl, qx, qy, outs, key, fit_ms, tick_ms, iters=50):
    """The node's steady state: the reference requests a new
    map on every spatial_data_size change (node.cpp:552-566) and the publisher
    adds one point per second (turtlesim_spatial_publisher.py:43), so the real
    per-change cost is a one-point sbo_append (block Cholesky update, the new
    row of L^-1, the last row block repacked) plus one full tick -- not the
    refit `end_to_end` prices.  `iters` appends of one point each (new points
    uniform over the training box, terrain.more_points), a full tick after
    each, the pair timed together; the context keeps the appended points."""
    import torch

    from safe_bayesian_optimization_amd.terrain import more_points
    ax, ay, aobs = more_points(wl, iters + 1, seed=2024)
    f32 = lambda v: torch.as_tensor(np.ascontiguousarray(v, np.float32), device=dev)  # noqa: E731
    AX, AY, AO = f32(ax), f32(ay), f32(aobs)

    def one(i):
        gm.append(AX[i:i + 1], AY[i:i + 1], AO[i:i + 1])
        gm.tick(qx, qy, wl.beta, wl.f_min, outputs=outs, key_out=key, async_=True)

    one(iters)     # warmup (the append path's code objects and buffers)
    torch.cuda.synchronize()
    t_app = 0.0
    t0 = time.perf_counter()
    for i in range(iters):
        t1 = time.perf_counter()
        gm.append(AX[i:i + 1], AY[i:i + 1], AO[i:i + 1])   # synchronous (the previous tick has finished)
        t_app += time.perf_counter() - t1
        gm.tick(qx, qy, wl.beta, wl.f_min, outputs=outs, key_out=key, async_=True)
        torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / iters
    m = qx.numel()
    return {"what": f"{iters} x (sbo_append of 1 point + a full tick) after the {wl.name} fit "
                    f"(N {wl.x.size} -> {wl.x.size + iters + 1})",
            "value": m / wall, "unit": "grid-points/s", "ms_per_step": wall * 1e3,
            "append_ms_avg": t_app * 1e3 / iters, "tick_ms_avg": wall * 1e3 - t_app * 1e3 / iters,
            "vs_refit_end_to_end": {"refit_plus_tick_ms": fit_ms + tick_ms,
                                    "speedup": (fit_ms + tick_ms) / (wall * 1e3)},
            "precise_sweep": gm.precision()[0], "n_after": gm.n}


def run_regime_stress(a, gm, prof, dev, n, gw, gh):
    """SURVEY.md 8(d) stress variant: the same N and grid size on the mapping
    node's own box [0, 1] x [0, 2.5] (config/lpsc.yaml:32-33), default plan:
    with l = 0.4 almost no tile is negligible.  Refits the context."""
    import torch

    from safe_bayesian_optimization_amd import _native as N
    from safe_bayesian_optimization_amd.terrain import synthetic_box
    wl = synthetic_box(n, gw, gh, seed=0, name=f"{a.config}-lpsc-box")
    f32 = lambda v: torch.as_tensor(np.ascontiguousarray(v, np.float32), device=dev)  # noqa: E731
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gm.fit(f32(wl.x), f32(wl.y), f32(wl.obs))
    torch.cuda.synchronize()
    fit_ms = (time.perf_counter() - t0) * 1e3
    qx, qy = f32(wl.qx), f32(wl.qy)
    m = qx.numel()
    key = torch.empty(2, dtype=torch.int64, device=dev)
    outs = dict(mu=torch.empty(m, dtype=torch.float32, device=dev), sd=torch.empty(m, dtype=torch.float32, device=dev),
                lo=torch.empty(m, dtype=torch.float64, device=dev), hi=torch.empty(m, dtype=torch.float64, device=dev),
                safe=torch.empty(m, dtype=torch.uint8, device=dev))

    def step():
        gm.tick(qx, qy, wl.beta, wl.f_min, score=N.SCORE_WIDTH, outputs=outs, key_out=key, async_=True)

    precise, perr, vmin, vmax = gm.precision()
    pinfo = gm.probe_info()
    pk = pinfo["precise_kernel"]
    res = _timed_ticks(prof, step, a.regime_steps)
    sd_default = outs["sd"].clone()
    # the other precise kernels on the same fit (the f64 MFMA sweep, and the
    # int8 sweep building K*'s digits itself when the default reads the K*
    # table): time and whole-grid variance difference
    others = {}
    if precise:
        for ok in ([0, 1] if pk == 3 else [0 if pk >= 1 else 1]):
            gm.set_option(N.SBO_OPT_PRECISE_KERNEL, ok)
            try:
                ores = _timed_ticks(prof, step, 1)
            finally:
                gm.set_option(N.SBO_OPT_PRECISE_KERNEL, pk)
            v_o = outs["sd"].double() ** 2
            v_d = sd_default.double() ** 2
            o = _regime_line(a, "lpsc_stress_box other precise kernel", f"SBO_OPT_PRECISE_KERNEL = {ok} on the same fit",
                             m, n, *ores, precise=True, precise_kernel=ok)
            o["variance_difference_vs_default"] = float((v_o - v_d).abs().max() / v_d.abs().max())
            o["default_speedup_over_this"] = o["ms_per_step"] / (res[0] * 1e3)
            others[ok] = o
    other = others.get(0)
    # the fast split sweep on the same fit, and its variance error against the
    # precise sweep over the whole grid (device against device; the tests
    # measure both against the fp64 oracle: tests/test_gpu_headline.py)
    gm.set_option(N.SBO_OPT_PRECISION, 0)
    try:
        fres = _timed_ticks(prof, step, 1)
    finally:
        gm.set_option(N.SBO_OPT_PRECISION, -1)
    v_def = sd_default.double() ** 2
    v_fast = outs["sd"].double() ** 2
    fast_err = float((v_fast - v_def).abs().max() / v_def.abs().max())
    fast = _regime_line(a, "lpsc_stress_box fast sweep", "SBO_OPT_PRECISION = 0 on the same fit", m, n, *fres)
    fast["variance_error_vs_precise_sweep"] = fast_err
    # the grid the node actually receives: the mapper's own resolution [300,
    # 120] over the same box (config/lpsc.yaml:34), the same
    # fit and default options -- the per-tick cost of the reference's path
    wm = synthetic_box(n, 300, 120, seed=0)
    mqx, mqy = f32(wm.qx), f32(wm.qy)
    mm = mqx.numel()
    mouts = dict(mu=torch.empty(mm, dtype=torch.float32, device=dev), sd=torch.empty(mm, dtype=torch.float32, device=dev),
                 lo=torch.empty(mm, dtype=torch.float64, device=dev), hi=torch.empty(mm, dtype=torch.float64, device=dev),
                 safe=torch.empty(mm, dtype=torch.uint8, device=dev))

    def mstep():
        gm.tick(mqx, mqy, wm.beta, wm.f_min, score=N.SCORE_WIDTH, outputs=mouts, key_out=key, async_=True)
    mres = _timed_ticks(prof, mstep, max(3, a.regime_steps))
    mapper = _regime_line(a, "lpsc_mapper_grid", "the same fit, the mapper's own 300 x 120 grid over the box "
                          "(config/lpsc.yaml:34), default options", mm, n, *mres, precise=precise, precise_kernel=pk)
    mapper["end_to_end"] = end_to_end(mm, fit_ms, mres[0] * 1e3)
    return _regime_line(a, "lpsc_stress_box", "N points and the grid on x [0, 1] x y [0, 2.5] (config/lpsc.yaml:32-33), "
                        "default options (SBO_OPT_PRECISION = -1: the fit-time probe picks the sweep)", m, n, *res,
                        extra={"fit_ms": fit_ms, "kstar_cutoff_log2": gm.skip_info()[0],
                               "end_to_end": end_to_end(m, fit_ms, res[0] * 1e3),
                               "precise_sweep": precise,
                               "precise_kernel": pk,
                               "inverse_check": gm.inverse_check(),
                               "probe": {"fast_sweep_variance_error": perr, "var_min": vmin, "var_max": vmax,
                                         "err_grid": pinfo["err_grid"], "err_train": pinfo["err_train"],
                                         "how": "32 x 32 grid over the training box + 512 training locations, "
                                                "fast vs precise sweep"},
                               "mapper_grid_300x120": mapper,
                               "other_precise_kernel": other,
                               "int8_in_sweep_kstar": others.get(1),
                               "fast_sweep": fast}, precise=precise, precise_kernel=pk)


def dtype_of(variant):
    return "f32 (bf16x3-split MFMA, f32 accumulation)" if variant in SPLIT_VARIANTS else "f32"


PEAK_F64_MFMA_TFLOPS = 78.6    # MI355X spec: dense FP64 matrix (v_mfma_f64_16x16x4_f64)
PEAK_I8_MFMA_TOPS = 5000.0     # MI355X_MICROARCH.md: i8 16x16x64 = 2x the bf16 rate per clock (dense)
OZ_PRODUCTS = 14               # predict_oz.hip: int8 digit-slice products per f64 product


def predict_roofline(variant, flops_f32, ms, mfma_flops, levels, precise=False, precise_kernel=1):
    """Roofline of the predictive kernel.  flops_f32 = the algorithmic work of
    one launch, 2*BM*BN*BK per multiplied k-tile (device counter); mfma_flops
    = the matrix-core work it issued (device counter: 2*BM*BN*BK per bf16
    MFMA product -- six per tile at full precision, three / one at the plan's
    reduced precision levels; one per tile for the f32 sweep), priced against
    the dense bf16 (split sweeps) or f32 peak."""
    f32_tf = flops_f32 / (ms * 1e-3) / 1e12
    ach = mfma_flops / (ms * 1e-3) / 1e12
    if precise and precise_kernel >= 1:
        tops = OZ_PRODUCTS * flops_f32 / (ms * 1e-3) / 1e12
        table = ("; K*'s digits from the K* table, built once per query block and k-tile, the queries in chunks "
                 "(plan + table + sweep per chunk, all in the time)" if precise_kernel == 3 else
                 "; K*'s digits built in the sweep")
        return {"kernel": "predict_oz_kernel (V = sf2 L^-1 K*^T from five A x four K* int8 digit slices: 14 "
                          "v_mfma_i32_16x16x64_i8 products per f64 product, exact int32 sums, f64 combination"
                          + table + ")",
                "bound": "mfma", "achieved": tops, "peak": PEAK_I8_MFMA_TOPS, "unit": "TOPS (int8)",
                "frac": tops / PEAK_I8_MFMA_TOPS, "int8_ops_per_launch": OZ_PRODUCTS * flops_f32,
                "algorithmic_flops_per_launch": flops_f32, "f64_equivalent_tflops": f32_tf,
                "f64_equivalent_over_f64_peak": f32_tf / PEAK_F64_MFMA_TFLOPS}
    if precise:
        return {"kernel": "predict_f64_kernel (V = sf2 L^-1 K*^T in f64: v_mfma_f64_16x16x4_f64, f64 K* and sums)",
                "bound": "mfma", "achieved": f32_tf, "peak": PEAK_F64_MFMA_TFLOPS, "unit": "TFLOP/s",
                "frac": f32_tf / PEAK_F64_MFMA_TFLOPS, "algorithmic_flops_per_launch": flops_f32}
    if variant in SPLIT_VARIANTS:
        return {"kernel": "predict_x3_kernel (V = sf2 L^-1 K*^T: bf16x3-split operands, up to six "
                          "v_mfma_f32_16x16x32_bf16 per f32 product, f32 accumulation)",
                "bound": "mfma", "achieved": ach, "peak": PEAK_BF16_MFMA_TFLOPS, "unit": "TFLOP/s",
                "frac": ach / PEAK_BF16_MFMA_TFLOPS, "mfma_flops_per_launch": mfma_flops,
                "algorithmic_flops_per_launch": flops_f32, "tiles_by_level_per_launch": levels,
                "f32_equivalent_tflops": f32_tf, "f32_equivalent_over_f32_peak": f32_tf / PEAK_F32_MFMA_TFLOPS}
    return {"kernel": "predict_kernel (V = sf2 L^-1 K*^T, f32 MFMA 16x16x4)", "bound": "mfma", "achieved": f32_tf,
            "peak": PEAK_F32_MFMA_TFLOPS, "unit": "TFLOP/s", "frac": f32_tf / PEAK_F32_MFMA_TFLOPS,
            "algorithmic_flops_per_launch": flops_f32}


def run_streaming(a, dev, world, rank):
    """C5: 50 iterations, N 1000 -> 8000 by sbo_append, 512x512 grid."""
    import torch

    from safe_bayesian_optimization_amd import TerrainMapper, synthetic
    from safe_bayesian_optimization_amd import _native as N
    from safe_bayesian_optimization_amd.dist import key_tensor_to_pairs
    if world != 1:
        raise SystemExit("C5 is a single-GPU streaming configuration")
    n_end, n0, iters, g = 8000, 1000, 50, a.grid or 512
    wl = synthetic(n_end, g, g, seed=0, name="C5")
    chunks = np.linspace(n0, n_end, iters + 1).round().astype(int)
    stream = torch.cuda.current_stream(dev)
    gm = TerrainMapper(dev.index, wl.hyper)
    gm.set_option(N.SBO_OPT_KERNEL_VARIANT, a.variant)
    gm.set_option(N.SBO_OPT_RESORT, a.resort)
    gm.ctx.set_stream(stream)
    prof = Prof(N.lib(), gm.ctx.handle)
    f32 = lambda v: torch.as_tensor(np.ascontiguousarray(v, np.float32), device=dev)  # noqa: E731
    X, Y, OBS = f32(wl.x), f32(wl.y), f32(wl.obs)
    qx, qy = f32(wl.qx), f32(wl.qy)
    m = qx.numel()
    outs = dict(mu=torch.empty(m, device=dev), sd=torch.empty(m, device=dev),
                lo=torch.empty(m, dtype=torch.float64, device=dev), hi=torch.empty(m, dtype=torch.float64, device=dev),
                safe=torch.empty(m, dtype=torch.uint8, device=dev))
    key = torch.empty(2, dtype=torch.int64, device=dev)

    def loop():
        gm.fit(X[:n0], Y[:n0], OBS[:n0])
        t_app = t_tick = 0.0
        last = None
        for i in range(iters):
            a0, a1 = chunks[i], chunks[i + 1]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            gm.append(X[a0:a1], Y[a0:a1], OBS[a0:a1])
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            gm.tick(qx, qy, wl.beta, wl.f_min, outputs=outs, key_out=key)
            last = key.cpu()
            t_tick += time.perf_counter() - t1
            t_app += t1 - t0
        return t_app, t_tick, last

    for _ in range(a.warmup):
        loop()
    prof.reset()
    reps = max(1, a.steps // iters)
    t0 = time.perf_counter()
    t_app = t_tick = 0.0
    last = None
    for _ in range(reps):
        ta, tt, last = loop()
        t_app += ta
        t_tick += tt
    elapsed = time.perf_counter() - t0
    pr = prof.read()
    prof.reset(False)
    steps = reps * iters
    pred_ms = pr["predict_ms"] / max(pr["predict_launches"], 1)
    flops = pr["predict_flops"] / max(pr["predict_launches"], 1)
    mflops = pr["mfma_flops"] / max(pr["predict_launches"], 1)
    levels = [x / max(pr["predict_launches"], 1) for x in pr["tiles_by_level"]]
    (s, i), = key_tensor_to_pairs(last)
    cpu = cpu_baseline_streaming(gm, wl, chunks, a.cpu_seconds) if not a.no_cpu else None
    value = m * steps / elapsed
    if cpu is not None:
        cpu["gpu_over_cpu"] = value / cpu["value"]
    traffic, traffic_src = pmc_traffic("C5", n_end, m, m)
    return {
        "metric": METRIC, "value": value, "unit": "grid-points/s", "n_gpus": 1, "steps": steps,
        "warmup": a.warmup, "ms_per_step": elapsed * 1e3 / steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": dtype_of(a.variant), "data": DATA,
        "config": {"workload": "C5", "n_train": [n0, n_end], "iterations": iters, "grid": [g, g], "M": m,
                   "parallelism": "single", "resort_pct": a.resort,
                   "step": "sbo_append (block Cholesky update; a k-d re-sort + refactor when the points appended "
                           "since the last sort exceed resort_pct %) + sbo_tick (includes one fit per loop)"},
        "roofline": dict(predict_roofline(a.variant, flops, pred_ms, mflops, levels), traffic=traffic,
                         traffic_source=traffic_src, avg_launch_ms=pred_ms),
        "append_ms_avg": t_app * 1e3 / steps, "tick_ms_avg": t_tick * 1e3 / steps,
        "argmax": {"index": i, "score": s}, "cpu_baseline": cpu,
    }


def cpu_baseline_streaming(gm, wl, chunks, budget_s):
    """C5's CPU comparator: the same Eigen-class dense path (cpu_baseline) on
    the host's `nproc` cores, per iteration an append (block Cholesky update:
    L21 by a triangular solve, K22 - L21 L21^T, its Cholesky; scipy/OpenBLAS)
    and a tick over the 512 x 512 grid.  Both are timed at the loop's last
    size (N 7857 -> 8000; the tick on a bounded sample of the grid,
    extrapolated linearly in M) and scaled to the loop's average by the mean
    of N^2 over the iterations (the tick's strsm and the append's solve are
    O(N^2) per query / per new point)."""
    import scipy.linalg as sla
    from threadpoolctl import threadpool_limits

    from oracle import oracle as O
    threads, total = host_cores()
    O.set_threads(threads)
    L, alpha = gm.factor()
    o = gm.order()
    h = wl.hyper
    n = L.shape[0]
    b = int(chunks[-1] - chunks[-2])
    n0 = n - b
    xs, ys = wl.x.astype(np.float32)[o], wl.y.astype(np.float32)[o]
    bp = O.BlasPredictor(L, alpha, xs, ys, h.length_scale, h.sf2, h.prior_mean)
    with threadpool_limits(limits=threads, user_api="blas"):
        # an append of b points on the CPU: the factor's last b rows against
        # its leading n0 x n0 block.  (With SBO_OPT_RESORT the factor's rows
        # are in k-d order after a re-sort, so these b rows are not the
        # caller's last batch but the same sizes: n0 x b solve, b x b update)
        L11 = np.ascontiguousarray(L[:n0, :n0])
        t0 = time.perf_counter()
        K22 = O.rbf_fill_f32in(xs[n0:], ys[n0:], h.length_scale, h.sf2, h.noise_level).astype(np.float32)
        Kx = np.empty((n0, b), np.float32, order="F")
        O.lib().orc_cross_kernel_f32(xs[:n0], ys[:n0], n0, xs[n0:], ys[n0:], b, h.length_scale, h.sf2,
                                     Kx.ctypes.data)
        L21t = sla.solve_triangular(L11, Kx, lower=True, check_finite=False)
        K22 -= L21t.T @ L21t
        sla.cholesky(K22.astype(np.float64), lower=True, check_finite=False)
        t_app = time.perf_counter() - t0
        k = bp.block
        bp.tick(wl.qx[:k], wl.qy[:k], wl.beta, wl.f_min)
        t0 = time.perf_counter()
        bp.tick(wl.qx[:k], wl.qy[:k], wl.beta, wl.f_min)
        t = time.perf_counter() - t0
        k2 = int(min(wl.qx.size, max(k, k * max(budget_s - 2 * t, 0.0) / max(t, 1e-6))))
        k2 = max(k, (k2 // k) * k)
        t0 = time.perf_counter()
        bp.tick(wl.qx[:k2], wl.qy[:k2], wl.beta, wl.f_min)
        t_tick = (time.perf_counter() - t0) * wl.qx.size / k2
    ns = np.asarray(chunks[1:], np.float64)
    scale = float(np.mean(ns ** 2) / float(n) ** 2)
    step_s = (t_app + t_tick) * scale
    return {"value": wl.qx.size / step_s, "unit": "grid-points/s", "cores": threads, "host_cpus": total,
            "kind": "port", "append_s_last": t_app, "tick_s_last": t_tick, "n2_scale": scale,
            "sample": f"last iteration sizes (N {n0} -> {n}; the factor's last {b} rows against its leading "
                      f"block, rows in k-d order after a re-sort): CPU block append + a dense tick over {k2} of the "
                      f"{wl.qx.size} grid points (oracle.BlasPredictor: OpenMP K*, sgemv, OpenBLAS strsm), "
                      f"extrapolated to the grid and scaled by mean(N_i^2)/N_last^2 = {scale:.3f} over the 50 "
                      f"iterations"}


def pmc_traffic(config, n, m_total, m):
    """HBM bytes per predict launch from the newest committed PMC summary of
    this config (tools/collect_pmc.sh: separate FETCH_SIZE / WRITE_SIZE
    rocprofv3 passes, gfx950 FETCH_SIZE x2), scaled to this rank's shard."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_{config}.json")))
    if not files or m_total == 0:
        return None, None
    try:
        d = json.load(open(files[-1]))
        t = d["predict_kernel"]["traffic_bytes"] * m / m_total
        return t, f"{os.path.relpath(files[-1], ROOT)} (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, separate passes)"
    except Exception:
        return None, None


GPUS_PER_NODE = 8   # an MI355X platform node: 8 OAM GPUs (the driver's SCALE node)


def host_cores():
    """Cores the CPU comparator may use: `nproc` (the CPUs this process may
    run on, honouring OMP_NUM_THREADS as GNU nproc does), and the machine's
    total beside it."""
    try:
        n = int(subprocess.run(["nproc"], capture_output=True, text=True, timeout=10).stdout.strip())
    except Exception:
        n = len(os.sched_getaffinity(0))
    return max(1, n), os.cpu_count() or n


def cpu_baseline(gm, wl, budget_s):
    """The Eigen-class dense CPU path on the host's cores: K*^T per query block
    (orc_cross_kernel_f32, OpenMP), mu by sgemv, V = L^-1 K*^T by OpenBLAS
    strsm (level-3, multithreaded), var, ComputeSets + argmax (oracle C), given
    the device's own factor; timed on a bounded contiguous sample of the grid
    and extrapolated linearly (the M axis is embarrassingly parallel).  Dense:
    it does not skip tiles -- the gpu_dense_over_cpu ratio compares like with
    like.  Timed at three thread counts: `nproc` (the
    box's OMP_NUM_THREADS share, the headline `value`), every CPU this process
    may run on (sched_getaffinity), and the per-GPU share of an 8-GPU node
    (host CPUs / 8).  Each count runs in a child process started with
    OMP_NUM_THREADS / OPENBLAS_NUM_THREADS set before numpy loads: OpenBLAS
    sizes its per-thread buffers for the thread count it starts with and
    crashes when raised past it at run time (measured: strsm with 10+ threads
    in a process that started with 8)."""
    import shutil
    import tempfile
    threads, total = host_cores()
    aff = len(os.sched_getaffinity(0))
    L, alpha = gm.factor()
    o = gm.order()                           # internal training order of the factor
    h = wl.hyper
    tmp = tempfile.mkdtemp(prefix="sbo_cpu_")
    try:
        np.save(os.path.join(tmp, "L.npy"), L)
        del L
        np.savez(os.path.join(tmp, "w.npz"), alpha=alpha, x=wl.x.astype(np.float32)[o], y=wl.y.astype(np.float32)[o],
                 qx=wl.qx, qy=wl.qy, p=np.array([h.length_scale, h.sf2, h.prior_mean, wl.beta, wl.f_min]))

        def child(nt, budget):
            env = dict(os.environ, OMP_NUM_THREADS=str(nt), OPENBLAS_NUM_THREADS=str(nt))
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-child", tmp,
                                "--cpu-seconds", str(budget)], env=env, capture_output=True, text=True,
                               timeout=max(120.0, 20 * budget))
            lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            if r.returncode != 0 or not lines:
                return {"threads": nt, "error": f"rc {r.returncode}: {r.stderr[-300:]}"}
            return json.loads(lines[-1])

        main = child(threads, budget_s)
        if "value" not in main:
            return None
        by = [dict(main, share="nproc (OMP_NUM_THREADS share of the box; the headline value)")]
        for nt, share in ((aff, "sched_getaffinity: every CPU this process may run on"),
                          (max(1, total // GPUS_PER_NODE), f"per-GPU share of an {GPUS_PER_NODE}-GPU node "
                                                           f"({total} host CPUs / {GPUS_PER_NODE})")):
            by.append(dict(child(nt, budget_s / 2) if nt != threads else main, share=share))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return {"value": main["value"], "unit": "grid-points/s", "cores": threads, "host_cpus": total,
            "affinity_cpus": aff, "kind": "port", "blas": main.get("blas"), "by_threads": by,
            "sample": f"{main['points']} contiguous grid points of {wl.name} (N={wl.x.size}): dense f32 K*^T "
                      f"(OpenMP) + sgemv mean + OpenBLAS strsm variance (oracle.BlasPredictor, the Eigen LLT-solve "
                      f"class) + ComputeSets + argmax, given the device L/alpha; {main['seconds']:.1f} s wall, "
                      f"extrapolated linearly; one child process per thread count"}


def cpu_child(path, budget):
    """bench.py --cpu-child DIR: one cpu_baseline measurement at the thread
    count this process was started with (OMP_NUM_THREADS)."""
    from threadpoolctl import threadpool_info

    from oracle import oracle as O
    nt = int(os.environ.get("OMP_NUM_THREADS", "1"))
    O.set_threads(nt)
    L = np.load(os.path.join(path, "L.npy"), mmap_mode="r")
    w = np.load(os.path.join(path, "w.npz"))
    ell, sf2, m0, beta, f_min = (float(v) for v in w["p"])
    bp = O.BlasPredictor(L, w["alpha"], w["x"], w["y"], ell, sf2, m0)
    del L
    qx, qy = w["qx"], w["qy"]

    def run(k):
        t0 = time.perf_counter()
        bp.tick(qx[:k], qy[:k], beta, f_min)
        return time.perf_counter() - t0

    blas = [f"{i.get('internal_api')} {i.get('version')} ({i.get('architecture')}, {i.get('num_threads')} threads)"
            for i in threadpool_info() if i.get("user_api") == "blas"]
    k = bp.block
    run(k)                                   # warm: thread pool, page-in of L
    t = run(k)
    k2 = int(min(qx.size, max(k, k * max(budget - 2 * t, 0.0) / max(t, 1e-6))))
    k2 = max(k, (k2 // k) * k)
    t2 = run(k2)
    print(json.dumps({"threads": nt, "value": k2 / t2, "points": k2, "seconds": t2, "blas": blas[0] if blas else None}),
          flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
