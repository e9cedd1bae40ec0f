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


class RankFailed(RuntimeError):
    """Raised on every rank when another rank's shard failed (that rank raises its own error)."""


def _check_status(status, err):
    """status: per-rank 0 (ok) / 1 (failed) from the gathered buffers.  Every rank raises when any
    failed: a rank's exception must not leave the others blocked in a later collective."""
    if err is not None:
        raise err
    bad = [r for r, v in enumerate(status) if v != 0]
    if bad:
        raise RankFailed(f"rank(s) {bad} failed in their shard (see their own error)")


def all_gather_device(buf: torch.Tensor, ws: int, group=None) -> torch.Tensor:
    """The RCCL collective of gather_fitness / sharded_rows: one all_gather_into_tensor of every
    rank's equal-shape device buffer -> [ws, *buf.shape] on the same device."""
    full = torch.empty((ws * buf.shape[0],) + tuple(buf.shape[1:]), dtype=buf.dtype, device=buf.device)
    dist.all_gather_into_tensor(full, buf.contiguous(), group=group)
    return full.view((ws,) + tuple(buf.shape))


def gather_fitness(local, P: int, per: int, group=None, err=None, check: bool = True) -> torch.Tensor:
    """All-gather fixed-size fitness shards (padded to `per`) and trim to [P].  Each rank's block
    carries one status word (local is None / err set when this rank's shard failed), so a failure
    anywhere raises on every rank after the one collective instead of leaving ranks blocked.
    check=False skips reading the status words back (no host synchronisation: bench.py's timed
    loop, whose launches cannot fail between the status checks it makes before timing)."""
    rank, ws = world()
    if ws == 1:
        if err is not None:
            raise err
        return local[:P]
    gloo = dist.get_backend(group) == "gloo"
    dev = torch.device("cpu") if gloo else (local.device if local is not None else local_device())
    buf = torch.full((per + 1,), float("inf"), dtype=torch.float32, device=dev)
    if local is not None:
        buf[: local.numel()] = local.to(dev)
    buf[per] = 0.0 if err is None else 1.0
    if gloo:  # CPU path: gloo takes host tensors, no all_gather_into_tensor
        parts = [torch.empty_like(buf) for _ in range(ws)]
        dist.all_gather(parts, buf, group=group)
        full = torch.stack(parts)
    else:
        full = all_gather_device(buf, ws, group)  # RCCL over xGMI
    if check or err is not None:
        _check_status(full[:, per].tolist(), err)
    return full[:, :per].reshape(-1)[:P]


def sharded_fitness(evaluate_shard: Callable[[int, int], torch.Tensor], P: int, group=None) -> torch.Tensor:
    """evaluate_shard(lo, hi) -> fitness of individuals [lo, hi) on this rank's device;
    returns the full [P] fitness on every rank (an exception on any rank raises on all)."""
    rank, ws = world()
    lo, hi, per = shard_bounds(P, ws, rank)
    if ws == 1:
        return evaluate_shard(lo, hi)[:P]
    try:
        local, err = evaluate_shard(lo, hi), None
    except Exception as e:  # noqa: BLE001 -- re-raised after the collective, on every rank
        local, err = None, e
    return gather_fitness(local, P, per, group, err)


def sharded_rows(compute: Callable[[int, int], Tuple["np.ndarray", "np.ndarray"]], n: int, row_shape: tuple,
                 group=None):
    """compute(lo, hi) -> (values [hi-lo] f32, rows [hi-lo, *row_shape] f32) of items [lo, hi)
    on this rank; returns the full (values [n], rows [n, ...]) on every rank.  Items are split
    into contiguous blocks like the population (shard_map's P('i'), gp.py:264-267 shard_optimise);
    one all-gather of the padded blocks (values and rows packed together, plus one status row: an
    exception on any rank -- a rank with an empty block included -- raises on all)."""
    import numpy as np
    rank, ws = world()
    if ws == 1:
        return compute(0, n)
    lo, hi, per = shard_bounds(n, ws, rank)
    err = None
    try:
        vals, rows = compute(lo, hi)
    except Exception as e:  # noqa: BLE001 -- re-raised after the collective, on every rank
        vals = rows = None
        err = e
    width = 1 + int(np.prod(row_shape))
    buf = np.zeros((per + 1, width), np.float32)
    m = hi - lo
    if m > 0 and err is None:
        buf[:m, 0] = np.asarray(vals, np.float32)
        buf[:m, 1:] = np.asarray(rows, np.float32).reshape(m, -1)
    buf[per, 0] = 0.0 if err is None else 1.0
    t = torch.from_numpy(buf)
    if dist.get_backend(group) == "gloo":
        parts = [torch.empty_like(t) for _ in range(ws)]
        dist.all_gather(parts, t, group=group)
        full = torch.stack(parts)
    else:  # RCCL: device buffers
        full = all_gather_device(t.to(local_device()), ws, group).cpu()
    full = full.numpy()
    _check_status(full[:, per, 0].tolist(), err)
    full = full[:, :per].reshape(ws * per, width)[:n]
    return full[:, 0].copy(), full[:, 1:].reshape(n, *row_shape).copy()
