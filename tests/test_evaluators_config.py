"""Evaluator configuration: solver/schedule validation mirrors of the reference constructors."""
import numpy as np
import pytest

import multitreegp_amd as mt
from multitreegp_amd.evaluators import rk4_schedule


class Dopri5:  # stand-in with diffrax's class name
    pass


def test_notebook_schedule():
    ts = np.arange(0, 50, 0.2, dtype=np.float32)  # DynamicPolicy.ipynb get_data
    assert rk4_schedule(ts, 0.05, 1000) == (996, 4, 250)


def test_rejects_adaptive_solver_and_noise():
    env = mt.Acrobot(0.05, 0.0)
    with pytest.raises(NotImplementedError):
        mt.DynamicEvaluator(env, 2, 0.05, solver=Dopri5())
    with pytest.raises(NotImplementedError):
        mt.DynamicEvaluator(mt.Acrobot(0.05, 0.1), 2, 0.05)  # obs_noise > 0
    ev = mt.DynamicEvaluator(env, 2, 0.05, solver="rk4")
    assert ev.max_fitness == 1e4 and ev.latent_size == 4 and ev.obs_size == 4


def test_schedule_errors():
    with pytest.raises(ValueError):
        rk4_schedule(np.array([0.0, 0.07, 0.14], np.float32), 0.05, 100)  # not a multiple of dt0
    with pytest.raises(ValueError):
        rk4_schedule(np.array([0.0, 0.1, 0.3], np.float32), 0.05, 100)  # non-uniform
    with pytest.raises(ValueError):
        rk4_schedule(np.arange(0, 10, 0.1, dtype=np.float32), 0.05, 10)  # max_steps
    with pytest.raises(NotImplementedError):
        rk4_schedule(np.array([5.0, 5.1, 5.2], np.float32), 0.05, 100)  # offset start breaks the mask


def test_program_specs_dynamic():
    ev = mt.DynamicEvaluator(mt.Acrobot(0, 0), 2, 0.05)
    specs, roles = ev.program_specs()
    # state equations see [y, a, u]; readout in the drift sees y = 0, u = 0; at saves u = 0
    assert specs == [(0, 7, 0), (1, 7, 0), (2, 7, 0b1001111), (2, 7, 0b1000000)]
    assert roles["prog_readout"] == 2 and roles["prog_readout_save"] == 3
