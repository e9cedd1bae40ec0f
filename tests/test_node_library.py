"""Node library numbering (gp.py:132-199) and the population sampler (initialization.py)."""
import numpy as np
import pytest

import multitreegp_amd as mt
from multitreegp_amd import _native as nat
from multitreegp_amd.sampling import create_map_b_to_d, sample_population
from helpers import CONTROL_OPS, SR_OPS


def test_dynamic_policy_opcode_table():
    lib = mt.NodeLibrary(CONTROL_OPS, [["y1", "y2", "y3", "y4", "a1", "a2", "u"], ["a1", "a2"]], [2, 1])
    # + 2, - 3, * 4, sin 5, cos 6, y1..y4 7..10, a1 11, a2 12, u 13
    expect = {"+": 2, "-": 3, "*": 4, "sin": 5, "cos": 6, "y1": 7, "y2": 8, "y3": 9, "y4": 10, "a1": 11,
              "a2": 12, "u": 13}
    assert lib.string_to_node == expect
    assert list(lib.slots) == [0, 0, 2, 2, 2, 1, 1, 0, 0, 0, 0, 0, 0, 0]
    assert lib.input_format == ["y1", "y2", "y3", "y4", "a1", "a2", "u"]
    assert lib.var_start == 7 and lib.n_funcs == 14
    assert list(lib.fn_codes) == [nat.FN_ZERO, nat.FN_ZERO, nat.FN_ADD, nat.FN_SUB, nat.FN_MUL, nat.FN_SIN,
                                  nat.FN_COS] + [nat.FN_VAR] * 7
    np.testing.assert_array_equal(lib.variable_array[:2], np.ones((2, 7)))
    np.testing.assert_array_equal(lib.variable_array[2], [0, 0, 0, 0, 1, 1, 0])


def test_duplicates_and_unknown_operators():
    lib = mt.NodeLibrary([("+", None, 2), ("+", None, 2), ("/", None, 2)], [["x0", "x1"]], [2])
    assert lib.string_to_node == {"+": 2, "/": 3, "x0": 4, "x1": 5}
    with pytest.raises(NotImplementedError):
        mt.NodeLibrary([("erf", None, 1)], [["x"]], [1])
    ext = mt.NodeLibrary([("exp", None, 1), ("log", None, 1), ("sqrt", None, 1), ("tanh", None, 1), ("abs", None, 1)],
                         [["x"]], [1])  # round 3: jnp's exp / log / sqrt / tanh / abs
    assert list(ext.fn_codes[2:7]) == [nat.FN_EXP, nat.FN_LOG, nat.FN_SQRT, nat.FN_TANH, nat.FN_ABS]
    with pytest.raises(ValueError):
        mt.NodeLibrary([("exp", None, 2)], [["x"]], [1])
    with pytest.raises(ValueError):
        mt.NodeLibrary([("sin", None, 2)], [["x"]], [1])


def test_map_b_to_d_depth3():
    # SURVEY.md §2.1 re-derivation: depth 3 -> [6 5 2 4 3 1 0]
    np.testing.assert_array_equal(create_map_b_to_d(3), [6, 5, 2, 4, 3, 1, 0])


@pytest.mark.parametrize("depth,N", [(4, 30), (10, 64)])
def test_sampler_layout_invariants(depth, N):
    lib = mt.NodeLibrary(CONTROL_OPS, [["y1", "y2", "y3", "y4", "a1", "a2", "u"], ["a1", "a2"]], [2, 1])
    pop = sample_population(0, lib, 60, 2, max_init_depth=depth, max_nodes=N)
    assert pop.shape == (2, 60, 3, N, 4) and pop.dtype == np.float32
    for tree_set in pop.reshape(-1, 3, N, 4):
        for t, tree in enumerate(tree_set):
            f = tree[:, 0].astype(int)
            nz = np.nonzero(f)[0]
            assert len(nz) > 0 and nz[0] == N - len(nz) and np.all(np.diff(nz) == 1)  # packed at the end
            for k in nz:
                ar = lib.slots[f[k]]
                if ar >= 1:
                    assert tree[k, 1] == k - 1  # first operand directly below (initialization.py:46)
                if ar == 2:
                    assert 0 <= tree[k, 2] < k - 1
                if ar == 0:
                    assert tree[k, 1] == -1 and tree[k, 2] == -1
                if f[k] >= lib.var_start:
                    assert lib.variable_array[t][f[k] - lib.var_start] == 1  # allowed variable only


@pytest.mark.parametrize("depth,N", [(4, 30), (10, 64), (16, 128)])
def test_batch_sampler_matches_tree_sampler_distribution(depth, N):
    """sample_population samples all trees of a position together (sample_trees_batch); its
    distribution must equal the per-tree restatement of initialization.py (sample_tree, which
    the mutations use): node-count mean and quantiles, opcode frequencies."""
    from multitreegp_amd.sampling import sample_tree
    lib = mt.NodeLibrary(CONTROL_OPS, [["y1", "y2", "y3", "y4", "a1", "a2", "u"]], [1])
    new = sample_population(3, lib, 4000, 1, max_init_depth=depth, max_nodes=N)[0, :, 0]
    rng = np.random.default_rng(4)
    m = create_map_b_to_d(depth)
    old = np.stack([sample_tree(rng, lib, lib.variable_array[0], depth, N, 1.0, m) for _ in range(4000)])
    cn, co = (new[..., 0] != 0).sum(1), (old[..., 0] != 0).sum(1)
    assert abs(cn.mean() - co.mean()) < 0.05 * co.mean()
    for q in (50, 90, 99):
        assert abs(np.percentile(cn, q) - np.percentile(co, q)) <= max(2.0, 0.1 * np.percentile(co, q))
    fn = np.bincount(new[..., 0].astype(int).ravel(), minlength=lib.n_funcs)[1:] / cn.sum()
    fo = np.bincount(old[..., 0].astype(int).ravel(), minlength=lib.n_funcs)[1:] / co.sum()
    np.testing.assert_allclose(fn, fo, atol=0.012)
    # the coefficient leaves carry N(0, 1) values, every other row value 0
    vals = new[..., 3][new[..., 0] == 1]
    assert abs(vals.mean()) < 0.05 and abs(vals.std() - 1.0) < 0.05
    assert np.all(new[..., 3][new[..., 0] != 1] == 0)
