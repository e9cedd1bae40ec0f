"""Host flattener (same code the flatten kernel runs) vs the oracle's row-order interpreter."""
import numpy as np
import pytest

import multitreegp_amd as mt
import progsim
from multitreegp_amd import _native as nat
from multitreegp_amd.sampling import sample_population
from oracle import oracle as orc
from helpers import CONTROL_OPS, SR_OPS


# the round-3 unary operators (node_library.SUPPORTED_OPERATORS): load + op, no fused forms
EXT_OPS = [("exp", None, 1, 0.1), ("log", None, 1, 0.1), ("sqrt", None, 1, 0.1), ("tanh", None, 1, 0.1),
           ("abs", None, 1, 0.1)]


def _lib(ext=False):
    return mt.NodeLibrary(SR_OPS + [("sin", None, 1), ("cos", None, 1)] + (EXT_OPS if ext else []),
                          [["x0", "x1", "x2", "x3"]], [3])


def _same(a, b):
    return a.view(np.uint32) == b.view(np.uint32) or (np.isnan(a) and np.isnan(b))


@pytest.mark.parametrize("ext", [False, True])
def test_reference_distribution_trees_bit_exact(ext):
    lib = _lib(ext)
    nl = lib.native()
    pop = sample_population(9, lib, 120, 1, max_init_depth=7, max_nodes=48)[0]
    rng = np.random.default_rng(0)
    for cand in pop:
        for tree in cand:
            prog, need = nat.flatten_tree_host(tree, nl, 4)
            assert need <= nat.STACK_MAX and len(prog) <= (tree[:, 0] != 0).sum()
            for _ in range(2):
                d = (rng.standard_normal(4) * 2).astype(np.float32)
                assert _same(progsim.run(prog, d), orc.eval_tree(tree, lib.fn_codes, lib.n_funcs, lib.var_start, d))


@pytest.mark.parametrize("ext", [False, True])
def test_garbage_arrays_follow_body_fun(ext):
    lib = _lib(ext)
    nl = lib.native()
    rng = np.random.default_rng(1)
    n = 0
    for _ in range(1500):
        N = int(rng.integers(1, 20))
        t = np.empty((N, 4), np.float32)
        t[:, 0] = rng.integers(-3, lib.n_funcs + 3, N) + (rng.random(N) < 0.1) * 0.5
        t[:, 1] = rng.integers(-N - 3, N + 3, N)
        t[:, 2] = rng.integers(-N - 3, N + 3, N)
        t[:, 3] = rng.standard_normal(N) * 3
        try:
            prog, _ = nat.flatten_tree_host(t, nl, 4, L=4096)
        except ValueError:
            continue
        d = rng.standard_normal(4).astype(np.float32)
        assert _same(progsim.run(prog, d), orc.eval_tree(t, lib.fn_codes, lib.n_funcs, lib.var_start, d)), t
        n += 1
    assert n > 1000


def test_zero_mask_folding_is_exact():
    """y/u slots known to be +0.0 (readout in dyn.py:113) fold to constants, bit-exactly."""
    lib = mt.NodeLibrary(CONTROL_OPS, [["y1", "y2", "y3", "y4", "a1", "a2", "u"], ["a1", "a2"]], [2, 1])
    nl = lib.native()
    pop = sample_population(2, lib, 200, 1, max_init_depth=6, max_nodes=40)[0]
    rng = np.random.default_rng(2)
    zmask = 0b1001111
    for cand in pop:
        tree = cand[0]
        prog, _ = nat.flatten_tree_host(tree, nl, 7, zmask)
        d = rng.standard_normal(7).astype(np.float32)
        d[[0, 1, 2, 3, 6]] = 0.0
        assert _same(progsim.run(prog, d), orc.eval_tree(tree, lib.fn_codes, lib.n_funcs, lib.var_start, d))


def test_constant_subtrees_fold_to_one_load():
    lib = _lib()
    nl = lib.native()
    c = lib.string_to_node
    t = np.array([[1, -1, -1, 2.0], [1, -1, -1, 3.0], [c["*"], 1, 0, 0], [c["sin"], 2, -1, 0]], np.float32)
    prog, need = nat.flatten_tree_host(t, nl, 4)
    assert [p[0] for p in prog] == ["LDC"] and need == 0
    assert np.float32(prog[0][2]).view(np.uint32) == orc.sincos(np.array([6.0], np.float32))[0][0].view(np.uint32)


def test_stack_limit_and_length_errors():
    """Row k = (+, k-1, k-1) is a DAG: postorder duplicates it, the stack need grows by one per
    row (Sethi-Ullman) and the program doubles -> MTGP_ERR_STACK / MTGP_ERR_PROG_TOO_LONG."""
    lib = _lib()
    nl = lib.native()
    add = lib.string_to_node["+"]
    rows = [[lib.string_to_node["x0"], -1, -1, 0]] + [[add, k - 1, k - 1, 0] for k in range(1, 11)]
    t = np.array(rows, np.float32)
    with pytest.raises(ValueError, match=str(-nat.ERR_STACK)):
        nat.flatten_tree_host(t, nl, 4, L=1 << 14)
    prog, need = nat.flatten_tree_host(t[:8], nl, 4, L=1 << 14)  # need 6: fine, but 191 instructions
    # emitted: len(k) = 2 len(k-1) + 1, len(1) = 2 -> 191; the 64 leaf pairs fuse -> 127
    assert need == 6 and len(prog) == 127 and sum(n == "VV_ADD" or n == "VVP_ADD" for n, _, _ in prog) == 64
    # the length cap applies to the program as emitted (before fusion)
    with pytest.raises(ValueError, match=str(-nat.ERR_PROG_TOO_LONG)):
        nat.flatten_tree_host(t[:8], nl, 4, L=64)


def test_extended_unary_ops_flatten_to_load_and_op():
    """exp / log / sqrt / tanh / abs over a leaf are two words (no fused forms), over a subtree one;
    constant subtrees fold with the same fp32 specs; the program JIT declines them (the population
    is then interpreted)."""
    from helpers import tree_from_expr
    lib = _lib(True)
    nl = lib.native()
    names = {}
    for op in ("exp", "log", "sqrt", "tanh", "abs"):
        prog, _ = nat.flatten_tree_host(tree_from_expr((op, "x1"), lib, 10), nl, 4)
        names[op] = [p[0] for p in prog]
        assert names[op] == ["LDV", op.upper()], names[op]
        prog, _ = nat.flatten_tree_host(tree_from_expr((op, ("+", "x0", "x2")), lib, 10), nl, 4)
        assert [p[0] for p in prog] == ["VV_ADD", op.upper()]
        c = np.float32(0.7)
        prog, _ = nat.flatten_tree_host(tree_from_expr(("*", (op, float(c)), "x3"), lib, 10), nl, 4)
        want = orc.unary(lib.fn_codes[lib.string_to_node[op]], np.array([c], np.float32))[0]
        assert len(prog) == 1 and prog[0][0] == "VC_MUL" and np.float32(prog[0][2]).view(np.uint32) == want.view(np.uint32)
    import ctypes
    for op in ("exp", "log", "sqrt", "tanh", "abs"):
        L = 28
        out = (nat.MtgpInstr * L)()
        need = ctypes.c_int32(0)
        t = np.ascontiguousarray(tree_from_expr((op, "x1"), lib, 10), np.float32)
        n = nat.load().mtgp_flatten_tree_host(t.ctypes.data, 10, ctypes.byref(nl), 4, 0, L, ctypes.addressof(out),
                                              ctypes.byref(need))
        assert n == 2
        # both translations take them (round 4: exp / log / tanh / sqrt are subroutine calls -- v_mov
        # v17, v8 + s_getpc / s_add / s_addc / s_swappc -- abs one inline v_and_b32 with a literal);
        # register mode: the data load v_mov v8, v1 (1 word) + the op + the return
        words = nat.load().mtgp_jit_translate_host_ex(ctypes.addressof(out), L, None, 0, 0)
        assert words == 1 + (2 if op == "abs" else 6) + 1, (op, words)
        assert nat.load().mtgp_jit_translate_host_ex(ctypes.addressof(out), L, None, 0, 1) > words
