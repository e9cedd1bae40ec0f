"""Population sharding across GPUs (one process per GPU, torch.distributed over RCCL).

Restates the reference's data parallelism (gp.py:255-262, 412-415): a 1-D mesh over the
flattened population axis, ``P('i')`` in, ``P('i')`` out, data replicated (``P(None)``).
Here: rank r evaluates the contiguous block ``[r*P/G, (r+1)*P/G)`` (P padded up to a multiple
of G), then ONE all-gather of the fp32 fitness shard gives every rank the full ``[P]`` vector
for the host-side argmin / evolution.  There is no other collective on the data path.
"""
from __future__ import annotations

import os
from typing import Callable, Tuple

import torch
import torch.distributed as dist


def local_device() -> torch.device:
    """This process's GPU: cuda:LOCAL_RANK under torchrun (one process per GPU), else the current
    device.  The engines bind to it, so ranks never share GPU 0 by accident."""
    lr = os.environ.get("LOCAL_RANK")
    if lr is not None:
        n = torch.cuda.device_count()
        return torch.device("cuda", int(lr) % max(n, 1))
    return torch.device("cuda", torch.cuda.current_device())


def world() -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_bounds(P: int, world_size: int, rank: int) -> Tuple[int, int, int]:
    """(lo, hi, per_rank) of rank's contiguous block; P is padded to per_rank * world_size."""
    per = (P + world_size - 1) // world_size
    lo = min(rank * per, P)
    hi = min(lo + per, P)
    return lo, hi, per


def gather_fitness(local: torch.Tensor, P: int, per: int, group=None) -> torch.Tensor:
    """All-gather fixed-size fitness shards (padded to `per`) and trim to [P]."""
    rank, ws = world()
    if ws == 1:
        return local[:P]
    if dist.get_backend(group) == "gloo":  # CPU path: gloo takes host tensors, no all_gather_into_tensor
        buf = torch.full((per,), float("inf"), dtype=local.dtype)
        buf[: local.numel()] = local.cpu()
        parts = [torch.empty_like(buf) for _ in range(ws)]
        dist.all_gather(parts, buf, group=group)
        return torch.cat(parts)[:P]
    buf = torch.full((per,), float("inf"), dtype=local.dtype, device=local.device)
    buf[: local.numel()] = local
    out = torch.empty((per * ws,), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, buf, group=group)  # RCCL over xGMI
    return out[:P]


def sharded_fitness(evaluate_shard: Callable[[int, int], torch.Tensor], P: int, group=None) -> torch.Tensor:
    """evaluate_shard(lo, hi) -> fitness of individuals [lo, hi) on this rank's device;
    returns the full [P] fitness on every rank."""
    rank, ws = world()
    lo, hi, per = shard_bounds(P, ws, rank)
    local = evaluate_shard(lo, hi)
    return gather_fitness(local, P, per, group)


def sharded_rows(compute: Callable[[int, int], Tuple["np.ndarray", "np.ndarray"]], n: int, row_shape: tuple,
                 group=None):
    """compute(lo, hi) -> (values [hi-lo] f32, rows [hi-lo, *row_shape] f32) of items [lo, hi)
    on this rank; returns the full (values [n], rows [n, ...]) on every rank.  Items are split
    into contiguous blocks like the population (shard_map's P('i'), gp.py:264-267 shard_optimise);
    one all-gather of the padded blocks (values and rows packed together)."""
    import numpy as np
    rank, ws = world()
    if ws == 1:
        return compute(0, n)
    lo, hi, per = shard_bounds(n, ws, rank)
    vals, rows = compute(lo, hi)
    width = 1 + int(np.prod(row_shape))
    buf = np.zeros((per, width), np.float32)
    m = hi - lo
    if m > 0:
        buf[:m, 0] = np.asarray(vals, np.float32)
        buf[:m, 1:] = np.asarray(rows, np.float32).reshape(m, -1)
    t = torch.from_numpy(buf)
    if dist.get_backend(group) == "gloo":
        parts = [torch.empty_like(t) for _ in range(ws)]
        dist.all_gather(parts, t, group=group)
        full = torch.cat(parts)
    else:  # RCCL: device buffers
        dev = local_device()
        full = torch.empty((per * ws, width), dtype=torch.float32, device=dev)
        dist.all_gather_into_tensor(full, t.to(dev), group=group)
        full = full.cpu()
    full = full.numpy()[:n]
    return full[:, 0].copy(), full[:, 1:].reshape(n, *row_shape).copy()
