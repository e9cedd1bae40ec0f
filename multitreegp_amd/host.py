"""ctypes binding of the native host library (include/mtgp_host.h, csrc/mtgp_evolve.cpp): the
evolution step of GeneticProgramming (gp.py:475-525) in C++ with OpenMP, so the host work of a
generation is milliseconds next to the GPU evaluation.  multitreegp_amd.genetic_operators is the
numpy restatement it is tested against (distributions and layout invariants)."""
from __future__ import annotations

import ctypes
import os
import weakref

import numpy as np

HOST_ABI_VERSION = 1
_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libmtgp_host.so")
_handle = None

_i32p = ctypes.POINTER(ctypes.c_int32)
_f64p = ctypes.POINTER(ctypes.c_double)
_f32p = ctypes.POINTER(ctypes.c_float)


class MtgpEvolveConfig(ctypes.Structure):
    _fields_ = [("n_funcs", ctypes.c_int32), ("slots", _i32p), ("n_ops", ctypes.c_int32), ("op_index", _i32p),
                ("op_prob", _f64p), ("var_start", ctypes.c_int32), ("n_vars", ctypes.c_int32), ("var_mask", _f32p),
                ("max_init_depth", ctypes.c_int32), ("coefficient_sd", ctypes.c_float),
                ("current_generation", ctypes.c_int32), ("migration_period", ctypes.c_int32),
                ("migration_size", ctypes.c_int32), ("tournament_size", ctypes.c_int32),
                ("elite_size", ctypes.c_int32), ("tournament_prob", _f64p), ("reproduction_type_prob", _f64p),
                ("reproduction_prob", _f64p)]


def load():
    """The host library; raises if it has not been built (__graft_entry__.build())."""
    global _handle
    if _handle is None:
        if not os.path.exists(_LIB):
            raise RuntimeError(f"{_LIB} missing: run __graft_entry__.build()")
        lib = ctypes.CDLL(_LIB)
        lib.mtgp_host_abi_version.restype = ctypes.c_int
        if lib.mtgp_host_abi_version() != HOST_ABI_VERSION:
            raise RuntimeError("libmtgp_host.so ABI mismatch: rebuild")
        lib.mtgp_evolve_populations.restype = ctypes.c_int
        lib.mtgp_evolve_populations.argtypes = [_f32p, _f32p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                                ctypes.c_int32, ctypes.POINTER(MtgpEvolveConfig), ctypes.c_uint64,
                                                _f32p]
        lib.mtgp_sample_population.restype = ctypes.c_int
        lib.mtgp_sample_population.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                               ctypes.POINTER(MtgpEvolveConfig), ctypes.c_uint64, _f32p]
        _handle = lib
    return _handle


def _ptr(a, t):
    return a.ctypes.data_as(t)


class _Lease:
    """Exports a pooled block (HostEvolver._output) as a fresh array; holds the block alive for as
    long as any array on it exists."""
    __slots__ = ("_block", "__array_interface__", "__weakref__")

    def __init__(self, block: np.ndarray):
        self._block = block
        self.__array_interface__ = {"data": (block.ctypes.data, False), "shape": block.shape, "typestr": "<f4",
                                    "version": 3}


class HostEvolver:
    """The library + strategy parameters packed once into an MtgpEvolveConfig (the arrays are kept
    alive by this object)."""

    def __init__(self, library, max_nodes: int, max_init_depth: int, coefficient_sd: float = 1.0,
                 migration_period: int = 10, migration_size: int = 0, tournament_size: int = 7, elite_size: int = 0,
                 tournament_probabilities=None, reproduction_type_probabilities=None,
                 reproduction_probabilities=None, num_populations: int = 1):
        self.lib = load()
        self._pool = []  # populations returned by evolve (see _output)
        self.N = int(max_nodes)
        self.num_populations = int(num_populations)
        self._slots = np.ascontiguousarray(library.slots, np.int32)
        self._ops = np.ascontiguousarray(library.operator_indices, np.int32)
        op_p = np.asarray(library.operator_probabilities, np.float64)
        self._op_p = np.ascontiguousarray(op_p / op_p.sum())
        vi = np.asarray(library.variable_indices)
        assert np.array_equal(vi, np.arange(vi[0], vi[0] + len(vi))), "variables must be contiguous indices"
        self._var_mask = np.ascontiguousarray(library.variable_array, np.float32)
        self.num_trees = self._var_mask.shape[0]
        P = self.num_populations
        tp = np.ones((P, tournament_size)) if tournament_probabilities is None else tournament_probabilities
        rtp = np.tile([1.0, 0.0, 0.0], (P, 1)) if reproduction_type_probabilities is None \
            else reproduction_type_probabilities
        rp = np.ones(P) if reproduction_probabilities is None else reproduction_probabilities
        self._tp = np.ascontiguousarray(np.asarray(tp, np.float64).reshape(P, tournament_size))
        self._rtp = np.ascontiguousarray(np.asarray(rtp, np.float64).reshape(P, 3))
        self._rp = np.ascontiguousarray(np.asarray(rp, np.float64).reshape(P))
        self.cfg = MtgpEvolveConfig(
            len(self._slots), _ptr(self._slots, _i32p), len(self._ops), _ptr(self._ops, _i32p),
            _ptr(self._op_p, _f64p), int(vi[0]), len(vi), _ptr(self._var_mask, _f32p), int(max_init_depth),
            float(coefficient_sd), 0, int(migration_period), int(migration_size), int(tournament_size),
            int(elite_size), _ptr(self._tp, _f64p), _ptr(self._rtp, _f64p), _ptr(self._rp, _f64p))

    @classmethod
    def for_strategy(cls, gp) -> "HostEvolver":
        """From a GeneticProgramming instance's parameters (gp.py:61-121)."""
        return cls(gp.library, gp.max_nodes, gp.max_init_depth, gp.coefficient_sd, gp.migration_period,
                   gp.migration_size, gp.tournament_size, gp.elite_size, gp.tournament_probabilities,
                   gp.reproduction_type_probabilities, gp.reproduction_probabilities, gp.num_populations)

    def evolve(self, populations, fitness, seed: int, current_generation: int) -> np.ndarray:
        pops = np.ascontiguousarray(populations, np.float32)
        fit = np.ascontiguousarray(fitness, np.float32)
        if pops.ndim != 5 or pops.shape[0] != self.num_populations or pops.shape[2:] != (self.num_trees, self.N, 4):
            raise ValueError(f"populations shape {pops.shape} does not match the strategy")
        if fit.shape != pops.shape[:2]:
            raise ValueError(f"fitness shape {fit.shape} does not match populations {pops.shape[:2]}")
        P, S = pops.shape[:2]
        pairs = (S - self.cfg.elite_size) // 2
        out = self._output((P, self.cfg.elite_size + 2 * pairs, self.num_trees, self.N, 4))
        self.cfg.current_generation = int(current_generation)
        rc = self.lib.mtgp_evolve_populations(_ptr(pops, _f32p), _ptr(fit, _f32p), P, S, self.num_trees, self.N,
                                              ctypes.byref(self.cfg), ctypes.c_uint64(seed & (2**64 - 1)),
                                              _ptr(out, _f32p))
        if rc < 0:
            raise ValueError("mtgp_evolve_populations rejected its arguments")
        return out

    def _output(self, shape) -> np.ndarray:
        """The array evolve writes: the memory of a population this object returned earlier that
        nothing references any more (the user's loop has moved on to a newer generation), else new
        memory.  A fresh 537 MB C5 population costs more in first-touch page faults than the whole
        evolution step; reusing dead memory keeps the reference's value semantics (no array the
        caller can still see is ever overwritten).

        Ownership, not reference counting: each returned array is built on a _Lease, a non-array
        object exporting the pooled block through __array_interface__.  numpy stops base collapsing
        at a non-array base, so every view, slice, reshape, memoryview or torch.from_numpy of the
        returned array keeps the array -- and through it the lease -- alive; the pool holds the
        block strongly and the lease only through a weakref, and reuses a block once its lease is
        gone."""
        for i, (block, lease) in enumerate(self._pool):
            if block.shape == shape and lease() is None:
                return self._lend(i, block)
        block = np.empty(shape, np.float32)
        self._pool.append((block, None))
        out = self._lend(len(self._pool) - 1, block)
        if len(self._pool) > 3:
            self._pool.pop(0)  # an outstanding lease keeps its block alive by itself
        return out

    def _lend(self, i: int, block: np.ndarray) -> np.ndarray:
        lease = _Lease(block)
        self._pool[i] = (block, weakref.ref(lease))
        out = np.asarray(lease)
        assert out.base is lease and out.ctypes.data == block.ctypes.data
        return out

    def sample_population(self, pop_size: int, seed: int) -> np.ndarray:
        out = np.empty((self.num_populations, pop_size, self.num_trees, self.N, 4), np.float32)
        rc = self.lib.mtgp_sample_population(self.num_populations, pop_size, self.num_trees, self.N,
                                             ctypes.byref(self.cfg), ctypes.c_uint64(seed & (2**64 - 1)),
                                             _ptr(out, _f32p))
        if rc < 0:
            raise ValueError("mtgp_sample_population rejected its arguments")
        return out
