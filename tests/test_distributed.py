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


def _gp_worker(rank, ws, port, q):
    """GeneticProgramming.evaluate_population on world_size 2 with the shard evaluator injected
    (CPU oracle): sharding, the gloo all-gather, reshape and best-so-far bookkeeping."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        q.put((rank, _gp_run()))
    finally:
        dist.destroy_process_group()


def _gp_run():
    """Two generations of evaluate_population (num_populations 3 x population_size 6, P = 18:
    not divisible by 4) with an oracle shard evaluator -> fitness, best_fitnesses, best_solutions."""
    from helpers import CONTROL_OPS, oracle_model, oracle_rollouts, static_setup
    from oracle import oracle as orc
    import multitreegp_amd as mt
    env, lib, ff, data, pop = static_setup(P=36, R=4, n_steps=20, seed=8)
    gp = mt.GeneticProgramming(2, 6, ff, CONTROL_OPS, [["y1", "y2", "y3", "y4"]], [1], num_populations=3,
                               size_parsinomy=0.5, migration_percentage=0.5, elite_percentage=0.0, verbose=False)
    d = ff.prepare(data)
    model, ro = oracle_model(ff, d, parsimony=0.5), oracle_rollouts(d)
    calls = []

    def shard(flat, lo, hi, data_):
        calls.append((lo, hi))
        if hi <= lo:
            return torch.empty(0)
        return torch.from_numpy(orc.evaluate(model, flat[lo:hi], lib, ro)["fitness"])

    gp._evaluate_shard = shard
    out = []
    for g in range(2):
        populations = pop[18 * g:18 * (g + 1)].reshape(3, 6, *pop.shape[1:])
        fit, back = gp.evaluate_population(populations, data)
        assert fit.shape == (3, 6) and back.shape == populations.shape
        gp.current_generation += 1
        out.append(fit.tobytes())
    return out, gp.best_fitnesses.tobytes(), gp.best_solutions.tobytes(), calls


@pytest.mark.parametrize("ws", [2])
def test_genetic_programming_evaluate_population_sharded(ws):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gp_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(ws))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want_fit, want_bf, want_bs, calls = _gp_run()  # unsharded (world size 1)
    assert calls == [(0, 18), (0, 18)]
    for r in range(ws):
        fits, bf, bs, rcalls = res[r]
        assert fits == want_fit and bf == want_bf and bs == want_bs
        assert rcalls == [(9 * r, 9 * r + 9)] * 2  # contiguous block per rank, gp.py:259 P('i')


def _opt_worker(rank, ws, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        q.put((rank, _opt_run()))
    finally:
        dist.destroy_process_group()


def _opt_run():
    """Generation 14 of a coefficient-optimising run (gp.py:418-422) with the shard evaluator and
    the shard optimiser injected (the CPU oracle's loss and gradients): the 50 best candidates
    are split over the ranks (shard_optimise, gp.py:264-267) and all-gathered."""
    from helpers import SR_OPS, oracle_model, oracle_rollouts, sr_setup
    from multitreegp_amd import coefficients as co
    from oracle import oracle as orc
    import multitreegp_amd as mt
    env, lib, ff, data, pop = sr_setup(P=60, R=4, n_save=9, save_every=2, h=0.05, depth=4, N=20, seed=9)
    gp = mt.GeneticProgramming(20, 60, ff, SR_OPS, [["x0", "x1"]], [2], max_nodes=20, size_parsinomy=0.01,
                               coefficient_optimisation=True, gradient_steps=3, verbose=False)
    gp.current_generation = 14
    d = ff.prepare(data)
    d["h"] = ff.dt0
    model, ro = oracle_model(ff, d), oracle_rollouts(d)

    class OracleOpt(co.CoefficientOptimiser):
        def __init__(self):
            pass

        def loss_and_grad(self, cands, data_, rows=None):
            loss, grad, rws = orc.sr_grad(model, cands, lib, ro)
            return loss, [grad[b, : len(r)].copy() for b, r in enumerate(rws)]

    sizes = []

    def opt_shard(cands, data_):
        sizes.append(len(cands))
        if len(cands) == 0:
            return np.zeros(0, np.float32), cands
        return OracleOpt().optimise(cands, data_, gp.gradient_steps, gp.optimiser)

    gp._evaluate_shard = lambda flat, lo, hi, data_, parsimony=None: (
        torch.empty(0) if hi <= lo else torch.from_numpy(
            orc.evaluate(dict(model, parsimony=gp.size_parsinomy if parsimony is None else parsimony),
                         flat[lo:hi], lib, ro)["fitness"]))
    gp._optimise_shard = opt_shard
    fit, back = gp.evaluate_population(pop[None], data)
    return fit.tobytes(), back.tobytes(), gp.best_fitnesses.tobytes(), sizes


def test_coefficient_optimisation_sharded():
    """the optimisation of the 50 best candidates is split over the ranks and
    all-gathered; fitness and population equal the single-process run bit for bit."""
    ws = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_opt_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(ws))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want_fit, want_pop, want_bf, sizes = _opt_run()
    assert sizes == [50]
    for r in range(ws):
        fit, back, bf, rsizes = res[r]
        assert fit == want_fit and back == want_pop and bf == want_bf
        assert rsizes == [25]


def _fail_worker(rank, ws, port, q, which):
    """rank 1 raises inside its shard (which = "fitness") or has an empty block and rank 0
    raises (which = "rows"): every rank must raise, none may block in the collective."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        try:
            if which == "fitness":
                def shard(lo, hi):
                    if rank == 1:
                        raise ValueError("shard failed on rank 1")
                    return torch.zeros(hi - lo)
                mdist.sharded_fitness(shard, 6)
            else:
                def rows(lo, hi):  # n = 1 item: rank 1's block is empty
                    if rank == 0:
                        raise NotImplementedError("rank 0 cannot optimise")
                    return np.zeros(hi - lo, np.float32), np.zeros((hi - lo, 2), np.float32)
                mdist.sharded_rows(rows, 1, (2,))
            q.put((rank, "returned"))
        except Exception as e:  # noqa: BLE001
            q.put((rank, type(e).__name__))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("which", ["fitness", "rows"])
def test_failure_on_one_rank_raises_on_all(which):
    """an exception on one rank (a rank with an empty block included) used to leave the
    others blocked in the all-gather; the gathered blocks now carry a status word."""
    ws = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fail_worker, args=(r, ws, port, q, which)) for r in range(ws)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(ws))
    for p in procs:
        p.join(timeout=60)
    bad = 1 if which == "fitness" else 0
    assert res[bad] == ("ValueError" if which == "fitness" else "NotImplementedError")
    assert res[1 - bad] == "RankFailed"
