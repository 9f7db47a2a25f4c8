"""Multi-GPU sharding of the grid sweep.

Grid rows are independent given (L, alpha): each rank fits the same
measurements (replicated fit, no communication), sweeps a contiguous block of
M/P query rows, and reduces its masked argmax to a 16-byte key
``(score f64, global index i64)``.  The only collective on the data path is
one RCCL all-gather of those keys over xGMI (P x 16 bytes, latency bound),
combined on every rank with ``sbo_key_combine`` semantics (highest score,
lowest global index on ties).  The key is 16 bytes rather than a packed u64
because the score is the node's f64 width Q(:,1)-Q(:,0) (node.cpp:516),
which does not fit beside an index in 64 bits without rounding.
"""
from __future__ import annotations

import struct

import numpy as np


def shard_range(m: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous row block [lo, hi) of rank ``rank`` (sizes differ by <= 1)."""
    base, rem = divmod(m, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def combine_keys(keys) -> tuple[float, int]:
    """Reduce (score, idx) pairs: highest score, lowest index on ties; idx -1 = none."""
    best_s, best_i = 0.0, -1
    for s, i in keys:
        i = int(i)
        if i < 0:
            continue
        if best_i < 0 or s > best_s or (s == best_s and i < best_i):
            best_s, best_i = float(s), i
    return best_s, best_i


def key_tensor_to_pairs(t) -> list[tuple[float, int]]:
    """(P, 2) int64 tensor/array of raw sbo_key bytes -> [(score, idx)]."""
    a = np.asarray(t.cpu() if hasattr(t, "cpu") else t, dtype=np.int64).reshape(-1, 2)
    return [(struct.unpack("<d", struct.pack("<q", int(r[0])))[0], int(r[1])) for r in a]


def allreduce_key(key_dev, group=None) -> tuple[float, int]:
    """All-gather each rank's 16-byte device key (RCCL on GPU tensors, gloo on
    CPU tensors) and combine."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    if world == 1:
        return combine_keys(key_tensor_to_pairs(key_dev))
    out = torch.empty(world * 2, dtype=torch.int64, device=key_dev.device)
    dist.all_gather_into_tensor(out, key_dev.reshape(2), group=group)
    return combine_keys(key_tensor_to_pairs(out))
