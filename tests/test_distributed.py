"""Population sharding + fitness all-gather (gp.py:255-262 restated), world_size 2 over gloo.

Each rank evaluates its contiguous block with an injected evaluator (the CPU oracle, as the
checker); the gathered fitness must equal the unsharded result bit-for-bit, including P not
divisible by the world size."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from multitreegp_amd import distributed as mdist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, P, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from helpers import oracle_model, oracle_rollouts, static_setup
        from oracle import oracle as orc
        env, lib, ff, data, pop = static_setup(P=P, R=4, n_steps=20, seed=5)
        d = ff.prepare(data)
        model, ro = oracle_model(ff, d), oracle_rollouts(d)

        def shard(lo, hi):
            if hi <= lo:
                return torch.empty(0)
            return torch.from_numpy(orc.evaluate(model, pop[lo:hi], lib, ro)["fitness"])

        full = mdist.sharded_fitness(shard, P).numpy()
        q.put((rank, full.tobytes()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("P", [10, 7])
def test_sharded_equals_unsharded(P):
    ws = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, P, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(ws))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from helpers import oracle_model, oracle_rollouts, static_setup
    from oracle import oracle as orc
    env, lib, ff, data, pop = static_setup(P=P, R=4, n_steps=20, seed=5)
    d = ff.prepare(data)
    want = orc.evaluate(oracle_model(ff, d), pop, lib, oracle_rollouts(d))["fitness"]
    for r in range(ws):
        got = np.frombuffer(res[r], np.float32)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_shard_bounds_cover():
    for P in (1, 7, 8, 8192, 65536):
        for ws in (1, 2, 4, 8):
            seen = []
            for r in range(ws):
                lo, hi, per = mdist.shard_bounds(P, ws, r)
                seen.extend(range(lo, hi))
                assert hi - lo <= per
            assert seen == list(range(P))
