"""GPU tests of the evaluation schedule (mtgp_schedule + MtgpRollouts.order).

The schedule only decides which individuals share a wave; every result must be bit-identical
to the unscheduled run and stay indexed by individual.  The schedule itself must be a
permutation that pairs expensive with cheap individuals (G >= 2) or runs the most expensive
first (G == 1)."""
import numpy as np
import pytest
import torch

from multitreegp_amd import _native as nat
from multitreegp_amd.engine import DeviceEngine
from helpers import bits_equal, dynamic_setup, sr_setup, static_setup

pytestmark = pytest.mark.gpu


def _costs(eng, fl):
    w = np.array(eng.schedule_weights(), dtype=np.int64)
    c = (eng.schedule_cost(fl).cpu().numpy().astype(np.int64) * w[None, :]).sum(axis=1)
    return np.clip(c, 0, nat.SCHED_BINS - 1)


# P up to 8192: the one-block schedule with the costs in registers; 9000: the one-block form that
# recomputes them (P * n_prog <= 65536 with 3 or 4 programs); 24000: histogram / scan / scatter in
# three launches
@pytest.mark.parametrize("P,R", [(P, R) for P in (1, 2, 7, 300) for R in (8, 32, 64)]
                         + [(8192, 32), (9000, 32), (9000, 64), (24000, 32), (24000, 64)])
def test_schedule_is_balanced_permutation(P, R):
    env, lib, ff, data, pop = dynamic_setup(P=P, R=R, n_steps=4, seed=3)
    eng = DeviceEngine(ff, lib, 0.0, "cuda:0")
    fl = eng.flatten(torch.from_numpy(pop).cuda())
    order = eng.schedule(fl, R).cpu().numpy()
    assert sorted(order.tolist()) == list(range(P))
    c = _costs(eng, fl)[order]
    if R == 64:  # G == 1: most expensive first
        assert np.all(np.diff(c) <= 0)
    else:
        h = P // 2
        hi, lo = c[0:2 * h:2], c[1:2 * h:2]
        assert np.all(np.diff(hi) <= 0) and np.all(np.diff(lo) >= 0) and np.all(hi >= lo)
        if P % 2:
            assert (hi.size == 0 or c[-1] <= hi.min()) and (lo.size == 0 or c[-1] >= lo.max())


def _eval(eng, pop_dev, data, **kw):
    res = eng.evaluate(pop_dev, data, trajectories=True, rollout_fitness=True, **kw)
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in res.items() if isinstance(v, torch.Tensor)}


def _same(a, b):
    assert a.keys() == b.keys()
    for k in a:
        assert bits_equal(a[k], b[k]), k


@pytest.mark.parametrize("setup,R", [(dynamic_setup, 8), (dynamic_setup, 32), (static_setup, 16), (sr_setup, 8)])
def test_schedule_does_not_change_results(setup, R):
    kw = dict(P=37, R=R) if setup is sr_setup else dict(P=37, R=R, n_steps=30)
    env, lib, ff, data, pop = setup(**kw)
    eng = DeviceEngine(ff, lib, 0.25, "cuda:0")
    pop_dev = torch.from_numpy(np.ascontiguousarray(pop)).cuda()
    plain = _eval(eng, pop_dev, data, schedule=False)
    _same(plain, _eval(eng, pop_dev, data, schedule=True))
    # an arbitrary permutation through MtgpRollouts.order
    fl = eng.flatten(pop_dev)
    fl.order = torch.from_numpy(np.random.default_rng(5).permutation(37).astype(np.int32)).cuda()
    _same(plain, _eval(eng, pop_dev, data, flattened=fl))


def test_schedule_rejects_bad_arguments():
    lib = nat.load()
    scratch = torch.empty((nat.SCHED_SCRATCH,), dtype=torch.int32, device="cuda:0")
    order = torch.empty((4,), dtype=torch.int32, device="cuda:0")
    plen = torch.ones((4, 2), dtype=torch.int32, device="cuda:0")
    w = (np.ctypeslib.ctypes.c_int32 * 2)(1, 1)
    for P, n_prog, R in ((4, 0, 8), (4, nat.MAX_PROGRAMS + 1, 8), (4, 2, 0), (4, 2, nat.MAX_ROLLOUTS + 1), (-1, 2, 8)):
        assert lib.mtgp_schedule(plen.data_ptr(), P, n_prog, w, R, order.data_ptr(), scratch.data_ptr(),
                                 None) == nat.ERR_ARG
