"""Node library: the opcode numbering of the reference (genetic_programming.py:132-199).

Opcodes: 0 = empty node, 1 = coefficient, 2 .. 2+K-1 = operators in ``operator_list`` order
(first occurrence of a name wins), then variables in first-appearance order over
``variable_list``.  ``slots`` is the arity per opcode and ``variable_array`` the per-tree mask
of allowed variables.  Operators are identified by NAME: the kernel implements the fixed set
``+ - * / sin cos`` (the reference's notebooks) and, since round 3, ``exp log sqrt tanh abs``
(jnp semantics in float32, specs in include/mtgp_f32math.h; the program JIT does not translate
these five, so a population using them runs in the interpreter); any other name is rejected
here, at construction, instead of failing inside the evaluator.
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import numpy as np

from . import _native as nat

# name -> (function code, arity)
SUPPORTED_OPERATORS = {
    "+": (nat.FN_ADD, 2),
    "-": (nat.FN_SUB, 2),
    "*": (nat.FN_MUL, 2),
    "/": (nat.FN_DIV, 2),
    "sin": (nat.FN_SIN, 1),
    "cos": (nat.FN_COS, 1),
    "exp": (nat.FN_EXP, 1),
    "log": (nat.FN_LOG, 1),
    "sqrt": (nat.FN_SQRT, 1),
    "tanh": (nat.FN_TANH, 1),
    "abs": (nat.FN_ABS, 1),
}


class NodeLibrary:
    """Mirror of the node-library part of ``GeneticProgramming.__init__``.

    :param operator_list: tuples ``(name, fn, arity[, probability])`` (gp.py:143-162)
    :param variable_list: one list of variable names per layer (gp.py:171-193)
    :param layer_sizes: trees per layer (gp.py:86, 95)
    """

    def __init__(self, operator_list: Sequence, variable_list: Sequence[Sequence[str]],
                 layer_sizes: Sequence[int]):
        layer_sizes = [int(x) for x in np.asarray(layer_sizes).reshape(-1)]
        self.operator_list = list(operator_list)  # the constructor arguments, kept for re-use
        self.variable_list = [list(v) for v in variable_list]
        assert len(operator_list) > 0, "No operators were given"
        assert len(layer_sizes) == len(variable_list), \
            "There is not a set of expressions for every type of layer"
        self.layer_sizes = layer_sizes
        self.num_trees = int(sum(layer_sizes))
        assert self.num_trees > 0, "The number of trees should be larger than 0"

        string_to_node: Dict[str, int] = {}
        node_to_string: Dict[int, str] = {}
        fn_codes: List[int] = [nat.FN_ZERO, nat.FN_ZERO]
        n_operands: List[int] = [0, 0]
        op_probs: List[float] = []
        index = 2
        for op in operator_list:
            name, arity = op[0], int(op[2])
            prob = float(op[3]) if len(op) == 4 else 1.0
            if name in string_to_node:
                continue
            if name not in SUPPORTED_OPERATORS:
                raise NotImplementedError(
                    f"operator {name!r} is not implemented by the MI355X kernel "
                    f"(supported: {sorted(SUPPORTED_OPERATORS)})")
            code, want = SUPPORTED_OPERATORS[name]
            if arity != want:
                raise ValueError(f"operator {name!r} has arity {want}, got {arity}")
            string_to_node[name] = index
            node_to_string[index] = name
            fn_codes.append(code)
            n_operands.append(arity)
            op_probs.append(prob)
            index += 1
        self.operator_indices = np.arange(2, index)
        self.operator_probabilities = np.asarray(op_probs, dtype=np.float32)
        var_start = index
        data_index = 0
        for var_list in variable_list:
            assert len(var_list) > 0, "An empty set of variables was given"
            for var in var_list:
                if var not in string_to_node:
                    string_to_node[var] = index
                    node_to_string[index] = var
                    fn_codes.append(nat.FN_VAR)
                    n_operands.append(0)
                    index += 1
                    data_index += 1
        if index > nat.MAX_FUNCS:
            raise ValueError(f"too many node functions ({index} > {nat.MAX_FUNCS})")
        self.var_start = var_start
        self.n_funcs = index
        self.n_variables = data_index
        self.variable_indices = np.arange(var_start, index)
        variable_array = np.zeros((self.num_trees, data_index), dtype=np.float32)
        counter = 0
        for layer_i, var_list in enumerate(variable_list):
            pmask = np.zeros(data_index, dtype=np.float32)
            for var in var_list:
                pmask[string_to_node[var] - var_start] = 1.0
            for _ in range(layer_sizes[layer_i]):
                variable_array[counter] = pmask
                counter += 1
        self.variable_array = variable_array
        self.slots = np.asarray(n_operands, dtype=np.int32)
        self.fn_codes = np.asarray(fn_codes, dtype=np.int8)
        self.string_to_node = string_to_node
        self.node_to_string = node_to_string

    @property
    def input_format(self) -> List[str]:
        """Variable order of the data vector (the reference prints it, gp.py:201)."""
        return [self.node_to_string[int(i)] for i in self.variable_indices]

    def native(self) -> nat.MtgpNodeLibrary:
        return nat.node_library_struct(self.n_funcs, self.var_start, self.fn_codes)

    # restatement of GeneticProgramming.tree_to_string (gp.py:310-328), used by tests
    def tree_to_string(self, tree: np.ndarray) -> str:
        tree = np.asarray(tree)
        if tree[-1, 0] == 1:
            return "{:.2f}".format(tree[-1, 3])
        elif tree[-1, 1] < 0:
            return self.node_to_string[int(tree[-1, 0])]
        elif tree[-1, 2] < 0:
            sub = self.tree_to_string(tree[: int(tree[-1, 1]) + 1])
            return f"{self.node_to_string[int(tree[-1, 0])]}({sub})"
        else:
            s1 = self.tree_to_string(tree[: int(tree[-1, 1]) + 1])
            s2 = self.tree_to_string(tree[: int(tree[-1, 2]) + 1])
            return f"({s1}){self.node_to_string[int(tree[-1, 0])]}({s2})"
