"""C4 (BASELINE config 4): the C3 workload at P = 65536, sharded over 8 GPUs.

The 8-GPU node is not ours to launch; this runs the C4 population at its real size through the
product's own sharding on one GPU: ``GeneticProgramming._evaluate_shard`` on every block
``shard_bounds(65536, 8, r)`` (the contiguous ``P('i')`` blocks of gp.py:255-262, 412-415) --
exactly what rank r evaluates under torchrun -- concatenated as the all-gather would, compared
bit for bit with one unsharded 65536-individual evaluation and, on a sample containing every
block boundary, with the CPU oracle.  The population is the bench's C4 workload: rank r's block
is the C3 population of seed 1000 + r (bench.setup_workload).
"""
import argparse
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from helpers import bits_equal, mismatch_report, oracle_model, oracle_rollouts  # noqa: E402

pytestmark = pytest.mark.gpu

WORLD = 8


def _c4_workload():
    import bench
    from multitreegp_amd.sampling import sample_population
    a = argparse.Namespace(config="c3", pop=8192, rollouts=32, ode_steps=200, solver="rk4", obs_noise=0.0)
    env, lib, ff, data, pop0 = bench.setup_workload(a, 0)
    blocks = [pop0] + [sample_population(1000 + r, lib, 8192, 1, max_init_depth=10, max_nodes=64)[0]
                       for r in range(1, WORLD)]
    return env, lib, ff, data, np.concatenate(blocks)


def test_c4_sharded_equals_unsharded_and_oracle():
    import torch
    from multitreegp_amd import distributed as mdist
    from multitreegp_amd.genetic_programming import GeneticProgramming
    from oracle import oracle as orc
    env, lib, ff, data, pop = _c4_workload()
    P = pop.shape[0]
    assert P == 65536
    gp = GeneticProgramming(1, P, ff, lib.operator_list, lib.variable_list, lib.layer_sizes, max_nodes=64,
                            migration_percentage=0.0, elite_percentage=0.0, device="cuda:0", verbose=False)
    shards, bounds = [], []
    for r in range(WORLD):
        lo, hi, per = mdist.shard_bounds(P, WORLD, r)
        assert per == 8192 and hi - lo == per
        shards.append(gp._evaluate_shard(pop, lo, hi, data).cpu().numpy())
        bounds.append((lo, hi))
    sharded = np.concatenate(shards)
    eng = gp._engine()
    whole = eng.evaluate(torch.from_numpy(pop).cuda(), data)["fitness"].cpu().numpy()
    assert bits_equal(sharded, whole), mismatch_report(sharded, whole, "C4 sharded vs unsharded")
    # the facade itself (world size 1 here: one shard) agrees too
    fit, _ = gp.evaluate_population(pop[None], data)
    assert bits_equal(fit.reshape(-1), whole)
    assert gp.best_fitnesses[0] == whole.min()
    # oracle sample: both ends of every block + random individuals (>= 64)
    pick = sorted({i for lo, hi in bounds for i in (lo, lo + 1, hi - 2, hi - 1)})
    rng = np.random.default_rng(4)
    pick += [int(i) for i in rng.choice(P, size=64, replace=False) if int(i) not in pick]
    idx = np.array(pick[:96])
    assert len(idx) >= 64
    d = eng.prepare_data(data)
    ref = orc.evaluate(oracle_model(ff, d), pop[idx], lib, oracle_rollouts(d))["fitness"]
    assert bits_equal(whole[idx], ref), mismatch_report(whole[idx], ref, "C4 vs oracle")
