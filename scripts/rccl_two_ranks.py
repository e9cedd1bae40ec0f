#!/usr/bin/env python3
"""The RCCL branches of multitreegp_amd.distributed on real hardware, two ranks (cuda:LOCAL_RANK
modulo the visible GPUs).  On a one-GPU box RCCL refuses two ranks on one device ("Duplicate GPU
detected", profiles/r05/v23_rccl2.log), so this needs a node with two or more GPUs:

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29531 scripts/rccl_two_ranks.py

Each rank checks gather_fitness / sharded_fitness / sharded_rows against the values it can
compute alone, and that a failure on one rank raises on both.  Prints one JSON line per rank."""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from multitreegp_amd import distributed as mdist  # noqa: E402


def main():
    rank, ws = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    assert dist.get_backend() == "nccl"
    out = {"rank": rank, "world": ws, "backend": dist.get_backend()}
    P = 1001
    full = torch.arange(P, dtype=torch.float32, device=dev) * 0.5
    lo, hi, per = mdist.shard_bounds(P, ws, rank)
    got = mdist.gather_fitness(full[lo:hi].clone(), P, per)
    out["gather_fitness"] = bool(torch.equal(got.cpu(), full.cpu()))
    got = mdist.sharded_fitness(lambda a, b: full[a:b].clone(), P)
    out["sharded_fitness"] = bool(torch.equal(got.cpu(), full.cpu()))
    rows = np.arange(P * 6, dtype=np.float32).reshape(P, 2, 3)
    vals, rr = mdist.sharded_rows(lambda a, b: (full[a:b].cpu().numpy(), rows[a:b]), P, (2, 3))
    out["sharded_rows"] = bool(np.array_equal(vals, full.cpu().numpy()) and np.array_equal(rr, rows))
    # a failure on one rank raises on both (no rank left blocked in a collective)
    try:
        def bad(a, b):
            if rank == 1:
                raise ValueError("deliberate")
            return full[a:b].clone()
        mdist.sharded_fitness(bad, P)
        out["failure_propagates"] = False
    except (ValueError, mdist.RankFailed) as e:
        out["failure_propagates"] = type(e).__name__
    dist.barrier()
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)
    ok = out["gather_fitness"] and out["sharded_fitness"] and out["sharded_rows"] and out["failure_propagates"]
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
