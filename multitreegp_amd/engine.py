"""Device engine: flatten a population and run the fused RK4 kernel through the C ABI.

PyTorch is used only as device-memory / stream plumbing (caching allocator, current HIP
stream); all compute is in libmtgp_hip.so.  The engine is the body of
``GeneticProgramming.evaluate_population`` (gp.py:403-433) and of the per-candidate
evaluator calls.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from . import _native as nat
from .node_library import NodeLibrary


def _require_gpu(device) -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("multitreegp_amd needs a ROCm GPU (MI355X); no CPU fallback exists")
    if device is None:
        from .distributed import local_device
        d = local_device()  # cuda:LOCAL_RANK under torchrun
    else:
        d = torch.device(device)
    if d.type != "cuda":
        raise ValueError(f"device {d} is not a GPU device")
    return d


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else int(t.data_ptr())


@dataclass
class Flattened:
    prog: torch.Tensor     # int32 [P, n_prog, L, 2]  (MtgpInstr)
    plen: torch.Tensor     # int32 [P, n_prog]
    nodes: torch.Tensor    # int32 [P]
    status: torch.Tensor   # int32 [P, n_prog]
    L: int
    n_prog: int
    order: Optional[torch.Tensor] = None  # int32 [P] evaluation schedule (mtgp_schedule)
    jit_words: Optional[torch.Tensor] = None  # int32 [P, n_prog] JIT code words per program (mtgp_flatten_ex)
    jit_cost: Optional[torch.Tensor] = None   # int32 [P, n_prog] schedule weight of the JIT code
    jit: Optional[tuple] = None           # (code ptr, offsets [units+1], info [3], capacity, chain) of the JIT
    jit_key: Optional[tuple] = None       # (R, order, engine id, chain, arena slot, arena generation) of that code
    order_lanes: Optional[int] = None     # lane set the schedule `order` was built for


class DeviceEngine:
    """Binds one fitness-function config + node library to the HIP kernels."""

    def __init__(self, fitness_function, library: NodeLibrary, size_parsinomy: float = 0.0, device=None,
                 native=None, jit: Optional[bool] = None, lanes: Optional[int] = None,
                 dp_budget: Optional[int] = None):
        """lanes: lanes per individual (MtgpRollouts.lanes); None = lane_set's occupancy policy,
        0 = R rounded up to a power of two (the densest packing), else at least that many.
        dp_budget: Dopri5 control models -- step attempts of the first of two launches
        (MtgpModel.dp_budget; 0 = one launch; None = MTGP_DP_BUDGET, else automatic: max_steps // 2,
        or one launch while the last two-launch evaluation parked few waves -- `_dp_choose`)."""
        self.lanes = lanes
        if dp_budget is None and os.environ.get("MTGP_DP_BUDGET"):
            dp_budget = int(os.environ["MTGP_DP_BUDGET"])
        self.dp_budget = None if dp_budget is None else int(dp_budget)
        self._dp_bufs = None
        self._dp_probe = None   # (event, pinned count, waves) of the last two-launch evaluation
        self._dp_frac = None    # its parked fraction
        self._dp_evals = 0
        self._dp_pinned = None
        self.ff = fitness_function
        self.lib = library
        self.parsimony = float(size_parsinomy)
        self.device = _require_gpu(device)
        self.native = native if native is not None else nat.load()
        self._node_lib = library.native()
        self._data_key = None
        self._data = None
        self._specs_dev = None
        self._specs_key = None
        # program JIT (csrc/mtgp_jit.h): on unless disabled here or by MTGP_JIT=0
        self.use_jit = (os.environ.get("MTGP_JIT", "1") != "0") if jit is None else bool(jit)
        self._arenas = [None, None]  # (pointer, bytes): a ring of two executable code buffers
        self._arena_i = 0
        self._arena_gen = [0, 0]     # bumped whenever a slot is (re)written: stale Flattened code is rebuilt
        self._jit_last = None        # (pinned host info, event, units) of a sampled build: capacity hint
        self._jit_builds = 0
        self._jit_bytes_per_unit = None  # learnt from earlier plans (None: estimate from G)
        self._grad_code = None  # (pointer, bytes): the coefficient optimiser's dual-code buffer

    def __del__(self):
        try:
            if any(a is not None for a in self._arenas) or self._grad_code is not None:
                torch.cuda.synchronize(self.device)
                for a in self._arenas + [self._grad_code]:
                    if a is not None:
                        self.native.mtgp_jit_free(a[0])
                self._arenas = [None, None]
                self._grad_code = None
        except Exception:
            pass

    def grad_code_buffer(self, nbytes: int):
        """The executable buffer of the coefficient optimiser's dual-number code (mtgp_ctl_grad_jit),
        grown when needed; every gradient call re-emits its code on the stream before the kernel."""
        if self._grad_code is None or self._grad_code[1] < nbytes:
            if self._grad_code is not None:
                torch.cuda.synchronize(self.device)
                self.native.mtgp_jit_free(self._grad_code[0])
                self._grad_code = None
            ptr = ctypes.c_void_p()
            rc = self.native.mtgp_jit_alloc(self.device.index or 0, nbytes, ctypes.byref(ptr))
            if rc != nat.OK or not ptr.value:
                raise RuntimeError(f"mtgp_jit_alloc({nbytes}) failed: {rc}")
            self._grad_code = (ptr.value, nbytes)
        return self._grad_code

    # ------------------------------------------------------------------ jit
    def _arena(self, nbytes: int):
        """Next buffer of the executable ring, grown when needed.  Alternating buffers keeps the code
        of the previous population untouched while a new one is written (stream-ordered)."""
        self._arena_i ^= 1
        self._arena_gen[self._arena_i] += 1
        a = self._arenas[self._arena_i]
        if a is None or a[1] < nbytes:
            if a is not None:
                torch.cuda.synchronize(self.device)
                self.native.mtgp_jit_free(a[0])
                self._arenas[self._arena_i] = None
            size = max(int(nbytes * 1.25) + 4096, 1 << 20)
            ptr = ctypes.c_void_p()
            rc = self.native.mtgp_jit_alloc(self.device.index or 0, size, ctypes.byref(ptr))
            if rc != nat.OK or not ptr.value:
                raise RuntimeError(f"mtgp_jit_alloc({size}) failed: {rc}")
            a = (ptr.value, size)
            self._arenas[self._arena_i] = a
        return a

    def jit_build(self, fl: Flattened, m, R: int, order: Optional[torch.Tensor]) -> Optional[tuple]:
        """Translate the flattened programs to machine code once (mtgp_jit_plan + mtgp_jit_emit)
        for lane set R (MtgpRollouts.lanes: 64 / R individuals per wave),
        without a host round trip: the buffer is sized from the code size per program seen in
        earlier builds (read back asynchronously), and the evaluator checks the plan's status and
        size on the device, interpreting when the code is unusable.  Returns None when disabled."""
        chain = self.jit_chain(m, fl.n_prog) if fl.jit_words is not None else nat.MtgpJitChain(0, 0, 0)
        key = (R, None if order is None else order.data_ptr(), id(self),
               (chain.next, chain.cond, chain.store, chain.put, chain.put_slot))
        if fl.jit_key is not None and fl.jit_key[:4] == key:
            slot, gen = fl.jit_key[4:]
            if slot is None or self._arena_gen[slot] == gen:  # code still in place (or none was built)
                return fl.jit
        fl.jit_key, fl.jit = key + (None, None), None
        if not self._jit_usable():
            return None
        if fl.jit_words is None and self._jit_mode() != nat.JIT_MODE_REGS:
            return None  # the translation-based plan/emit only build register-data code
        P = fl.prog.shape[0]
        n = self.native.mtgp_jit_units(P, fl.n_prog, R)
        if n < 0:
            return None
        optr = None if order is None else order.data_ptr()
        if self._jit_last is not None and self._jit_last[1].query():  # previous readback done: learn its size
            err, total = (int(v) for v in self._jit_last[0].tolist())
            if err == 0 and self._jit_last[2] > 0:
                self._jit_bytes_per_unit = total / self._jit_last[2] * 1.5
            self._jit_last = None
        offs = torch.empty((n + 1,), dtype=torch.int32, device=self.device)
        info = torch.empty((2,), dtype=torch.int32, device=self.device)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        if fl.jit_words is not None:  # sizes from the flatten pass
            rc = self.native.mtgp_jit_plan_words_chain(fl.jit_words.data_ptr(), P, fl.n_prog, R, optr,
                                                       ctypes.byref(chain), offs.data_ptr(), info.data_ptr(), stream)
        else:  # flattened without the sizing outputs: translate to size
            rc = self.native.mtgp_jit_plan(fl.prog.data_ptr(), P, fl.n_prog, fl.L, R, optr, offs.data_ptr(),
                                           info.data_ptr(), stream)
        if rc != nat.OK:
            raise RuntimeError(f"mtgp_jit_plan failed: {rc}")
        self._jit_builds += 1
        if self._jit_last is None and (self._jit_bytes_per_unit is None or self._jit_builds % 8 == 0):
            # asynchronous readback of the plan's code size (every 8th build once learned: the
            # device checks the capacity itself, this only tunes the arena estimate)
            host = torch.empty((2,), dtype=torch.int32, pin_memory=True)
            host.copy_(info, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._jit_last = (host, ev, n)
        G = max(1, 64 // (1 << max(R - 1, 0).bit_length()))
        per_unit = self._jit_bytes_per_unit or 1024.0 * G
        ptr, size = self._arena(int(n * per_unit) + 4096)
        if fl.jit_words is not None:
            rc = self.native.mtgp_jit_emit_words_chain(fl.prog.data_ptr(), fl.jit_words.data_ptr(), P, fl.n_prog,
                                                       fl.L, R, optr, ctypes.byref(chain), offs.data_ptr(), ptr, size,
                                                       self._jit_mode(), stream)
        else:
            rc = self.native.mtgp_jit_emit(fl.prog.data_ptr(), P, fl.n_prog, fl.L, R, optr, offs.data_ptr(), ptr,
                                           size, stream)
        if rc != nat.OK:
            raise RuntimeError(f"mtgp_jit_emit failed: {rc}")
        fl.jit = (ptr, offs, info, size, chain)
        fl.jit_key = key + (self._arena_i, self._arena_gen[self._arena_i])
        return fl.jit

    def jit_chain(self, m, n_prog: int) -> "nat.MtgpJitChain":
        """The role chain the evaluator of model struct `m` calls (mtgp_jit_chain); none when
        MTGP_JIT_CHAIN=0 (A/B switch) or in LDS-data mode."""
        ch = nat.MtgpJitChain(0, 0, 0)
        if os.environ.get("MTGP_JIT_CHAIN", "1") == "0":
            return ch
        if self._jit_mode() == nat.JIT_MODE_LDS and self.ff.model_id != nat.MODEL_SR:
            return ch  # (the runtime-state-size control kernels call one unit per program)
        rc = self.native.mtgp_jit_chain(ctypes.byref(m), n_prog, ctypes.byref(ch))
        if rc != nat.OK:
            raise RuntimeError(f"mtgp_jit_chain failed: {rc}")
        return ch

    @staticmethod
    def jit_ok(fl: Flattened) -> bool:
        """Whether the evaluations of `fl` ran JIT code (synchronises; tests and tooling)."""
        if fl.jit is None:
            return False
        err, total = (int(v) for v in fl.jit[2][:2].cpu().tolist())
        return err == 0 and 0 < total <= fl.jit[3]

    # ------------------------------------------------------------------ data
    @staticmethod
    def _host_array(x) -> np.ndarray:
        if isinstance(x, torch.Tensor):
            x = x.detach().cpu().numpy()
        return np.ascontiguousarray(np.asarray(x))

    @staticmethod
    def data_fingerprint(data) -> tuple:
        """Content key of a reference data tuple: shape, dtype and a 128-bit blake2b hash of every
        array in full (nested tuples such as `params` included; torch tensors, CUDA ones too, read
        back), so an array mutated in place anywhere is re-uploaded.  Hashing runs at
        about 1 GB/s: ~0.4 ms for the C5 ground truth, microseconds for rollout data."""
        import hashlib

        def fp(x):
            if isinstance(x, (tuple, list)):
                return ("seq", tuple(fp(y) for y in x))
            if x is None:
                return None
            a = np.ascontiguousarray(DeviceEngine._host_array(x))
            return (a.shape, a.dtype.str, hashlib.blake2b(a.reshape(-1).view(np.uint8), digest_size=16).digest())

        return fp(data)

    def prepare_data(self, data) -> dict:
        """Upload the reference data tuple once (cached on its content, see data_fingerprint)."""
        from . import prng
        key = (self.data_fingerprint(data), prng.prng_impl_code())
        if self._data is not None and key == self._data_key:
            return self._data
        host = self.ff.prepare(data)
        dev = {}
        for name in ("x0", "params", "targets", "ts", "ys_true", "obs_keys", "obs_w", "fit_kof"):
            a = host.get(name)
            a = None if a is None else np.asarray(a)
            dev[name] = None if a is None or a.size == 0 else torch.from_numpy(np.ascontiguousarray(a)).to(self.device)
        host.update({f"{k}_dev": v for k, v in dev.items()})
        self._data, self._data_key = host, key
        return host

    def _specs(self):
        specs, roles = self.ff.program_specs()
        n_data = self.ff.n_data()
        if n_data < self.lib.n_variables:
            # the reference fails too: lambda_leaf(i) indexes past the data vector (gp.py:30-31)
            raise IndexError(f"data vector has {n_data} entries but the node library defines "
                             f"{self.lib.n_variables} variables")
        key = tuple(specs)
        if key != self._specs_key:
            arr = (nat.MtgpProgramSpec * len(specs))()
            for i, sp in enumerate(specs):  # (tree, n_data, zero_mask[, gap_at, gap])
                arr[i].tree, arr[i].n_data, arr[i].zero_mask = sp[:3]
                arr[i].gap_at, arr[i].gap = sp[3:5] if len(sp) >= 5 else (0, 0)
            buf = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(self.device)
            self._specs_dev, self._specs_key = buf, key
        return specs, roles

    # -------------------------------------------------------------- flatten
    def flatten(self, pop: torch.Tensor) -> Flattened:
        """pop: float32 [P, T, N, 4] on the device."""
        P, T, N, four = pop.shape
        if four != 4:
            raise ValueError("population rows must have 4 columns [f, a, b, value]")
        if N > nat.MAX_NODES:
            raise ValueError(f"max_nodes {N} > {nat.MAX_NODES}")
        specs, _ = self._specs()
        for sp in specs:
            t = sp[0]
            if t >= T:
                raise ValueError(f"candidate has {T} trees, the evaluator needs tree {t}")
        n_prog = len(specs)
        L = self.program_stride(N)
        dev = self.device
        # one spare 32-byte block after the last program: a block prefetch never leaves the buffer
        prog_buf = torch.empty((P * n_prog * L * 2 + 8,), dtype=torch.int32, device=dev)
        prog = prog_buf[: P * n_prog * L * 2].view(P, n_prog, L, 2)
        plen = torch.empty((P, n_prog), dtype=torch.int32, device=dev)
        nodes = torch.empty((P,), dtype=torch.int32, device=dev)
        status = torch.empty((P, n_prog), dtype=torch.int32, device=dev)
        jw = jc = None
        if self._jit_usable():  # size the JIT translation in the same pass
            jw = torch.empty((P, n_prog), dtype=torch.int32, device=dev)
            jc = torch.empty((P, n_prog), dtype=torch.int32, device=dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        pop = pop if pop.data_ptr() % 16 == 0 else pop.clone()
        rc = self.native.mtgp_flatten_ex(pop.data_ptr(), P, T, N, ctypes.byref(self._node_lib),
                                         self._specs_dev.data_ptr(), n_prog, L, prog.data_ptr(),
                                         plen.data_ptr(), nodes.data_ptr(), status.data_ptr(), _ptr(jw), _ptr(jc),
                                         self._jit_mode(), stream)
        if rc != nat.OK:
            raise RuntimeError(f"mtgp_flatten failed: {rc}")
        return Flattened(prog, plen, nodes, status, L, n_prog, jit_words=jw, jit_cost=jc)

    @staticmethod
    def program_stride(N: int) -> int:
        """Program slot L for max_nodes N: 2N + 7 instructions + END, rounded up to a multiple of 4
        (the evaluators fetch four instructions per scalar load, mtgp.h)."""
        return (2 * N + 8 + 3) // 4 * 4

    def _jit_usable(self) -> bool:
        """The program JIT serves every kernel: data vector in v0-v7 (control models, SR with
        n_var <= 4) or in the wide SR kernel's LDS stage vector (mtgp_jit.h kJitModeLds)."""
        if not self.use_jit:
            return False
        if getattr(self.ff, "state_size", 0) > 3:  # runtime state sizes: LDS-data code, fixed-step kernels only
            return self.ff.solver_kind != "dopri5"
        return self.ff.n_data() <= 8 or self._jit_mode() == nat.JIT_MODE_LDS

    def _jit_mode(self) -> int:
        """LDS-data code for the wide-state SR kernel (n_var > 4), register-data code otherwise."""
        if self.ff.model_id == nat.MODEL_SR and self.ff.n_data() > 4:
            return nat.JIT_MODE_LDS
        if getattr(self.ff, "state_size", 0) > 3:  # the runtime-state-size kernels' LDS data vector (round 6)
            return nat.JIT_MODE_LDS
        return nat.JIT_MODE_REGS

    @staticmethod
    def check_status(fl: Flattened):
        worst = int(fl.status.max().item()) if fl.status.numel() else 0
        if worst == nat.ERR_PROG_TOO_LONG:
            raise ValueError("a tree flattens to more than 2*max_nodes+7 instructions (shared sub-DAGs?)")
        if worst == nat.ERR_STACK:
            raise ValueError(f"a tree needs more than {nat.STACK_MAX} operand-stack slots")
        if worst != 0:
            raise RuntimeError(f"flatten status {worst}")

    # ------------------------------------------------------------- schedule
    def schedule_weights(self) -> list:
        """Relative run count of each program per RK4 step (cost model of mtgp_schedule)."""
        specs, roles = self._specs()
        w = [4] * len(specs)  # state equations and the drift readout run in all 4 stages
        if roles["prog_readout_save"] != roles["prog_readout"]:
            w[roles["prog_readout_save"]] = 1  # once per save point
        return w

    def schedule_cost(self, fl: Flattened) -> torch.Tensor:
        """Per-program cost [P, n_prog] the schedule balances: the executed JIT code size when the
        programs run as JIT code (sin/cos dominate there), the program length otherwise."""
        if not self._jit_usable():
            return fl.plen
        if fl.jit_cost is not None:
            return fl.jit_cost
        P = fl.plen.shape[0]
        cost = torch.empty_like(fl.plen)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        rc = self.native.mtgp_jit_cost(fl.prog.data_ptr(), fl.plen.data_ptr(), P, fl.n_prog, fl.L, cost.data_ptr(),
                                       stream)
        if rc != nat.OK:
            raise RuntimeError(f"mtgp_jit_cost failed: {rc}")
        return cost

    def schedule(self, fl: Flattened, R: int) -> torch.Tensor:
        """Build (once per flattened population and lane set R) the wave schedule that balances
        per-wave work."""
        if fl.order is not None and fl.order_lanes != R:
            fl.order = None
        if fl.order is None:
            P = fl.plen.shape[0]
            order = torch.empty((P,), dtype=torch.int32, device=self.device)
            scratch = torch.empty((nat.SCHED_SCRATCH,), dtype=torch.int32, device=self.device)
            w = self.schedule_weights()
            wts = (ctypes.c_int32 * len(w))(*w)
            stream = torch.cuda.current_stream(self.device).cuda_stream
            cost = self.schedule_cost(fl)
            rc = self.native.mtgp_schedule(cost.data_ptr(), P, fl.n_prog, wts, R, order.data_ptr(),
                                           scratch.data_ptr(), stream)
            if rc != nat.OK:
                raise RuntimeError(f"mtgp_schedule failed: {rc}")
            fl.order = order
            fl.order_lanes = R
        return fl.order

    # ----------------------------------------------------------------- eval
    def model_struct(self, d: dict) -> "nat.MtgpModel":
        """MtgpModel of this evaluator config for prepared data `d` (prepare_data)."""
        _, roles = self._specs()
        m = nat.MtgpModel()
        m.model = self.ff.model_id
        m.n_var = d.get("n_var", 4)
        m.state_size = getattr(self.ff, "state_size", 0)
        env = getattr(self.ff, "env", None)
        m.n_obs = env.n_obs if env is not None else 0
        m.n_control = env.n_control if env is not None else 0
        m.n_targets = env.n_targets if env is not None else 0
        m.n_steps, m.save_every, m.n_save = d["n_steps"], d["save_every"], d["n_save"]
        m.h = self.ff.dt0
        m.max_fitness = self.ff.max_fitness
        m.parsimony = self.parsimony
        m.prog_state, m.prog_readout = roles["prog_state"], roles["prog_readout"]
        m.prog_readout_save, m.readout_save_same = roles["prog_readout_save"], roles["readout_save_same"]
        m.prng_impl = d.get("prng_impl", 0)
        m.env = d.get("env", nat.ENV_ACROBOT)
        m.solver, m.max_steps = d.get("solver", nat.SOLVER_RK4), d.get("max_steps", 0)
        m.rtol, m.atol, m.dtmin, m.dtmax = d.get("rtol", 0.0), d.get("atol", 0.0), d.get("dtmin", 0.0), d.get("dtmax", 0.0)
        for f in ("pid_custom", "pid_c1", "pid_c2", "pid_c3", "pid_safety", "pid_factormin", "pid_factormax",
                  "no_force_dtmin"):
            setattr(m, f, d.get(f, 0))
        return m

    def rollouts_struct(self, d: dict, P: Optional[int] = None) -> "nat.MtgpRollouts":
        """MtgpRollouts over the device copies of prepared data `d` (no schedule); lanes per
        individual from lane_set(P, R) when P is given (else R rounded up to a power of two)."""
        ro = nat.MtgpRollouts()
        ro.x0, ro.params, ro.targets = _ptr(d["x0_dev"]), _ptr(d["params_dev"]), _ptr(d["targets_dev"])
        ro.ts, ro.ys_true, ro.R = _ptr(d["ts_dev"]), _ptr(d["ys_true_dev"]), d["R"]
        ro.obs_keys, ro.obs_w = _ptr(d.get("obs_keys_dev")), _ptr(d.get("obs_w_dev"))
        ro.lanes = self.lane_set(P, d["R"]) if P is not None else 0
        ro.fit_kof = _ptr(d.get("fit_kof_dev"))
        return ro

    def _simds(self) -> int:
        if not hasattr(self, "_n_simds"):
            self._n_simds = 4 * torch.cuda.get_device_properties(self.device).multi_processor_count
        return self._n_simds

    def lane_set(self, P: int, R: int) -> int:
        """Lanes per individual (MtgpRollouts.lanes): R rounded up to a power of two, widened
        (fewer individuals per wave, so fewer program calls per wave) while the launch would have
        fewer waves than the GPU has SIMDs -- a wave alone on its SIMD runs at the same speed with
        one individual's programs as with several, so at small P.R the spare SIMDs take the other
        individuals instead (C2: 1024 x 16 rollouts -> 1024 waves of one individual instead of
        256 waves of four).  MTGP_LANES overrides (A/B).  Results do not depend on the choice."""
        Rp = 1 << max(R - 1, 0).bit_length()
        if self.lanes is not None:
            return max(Rp, 1 << max(int(self.lanes) - 1, 0).bit_length())
        env = os.environ.get("MTGP_LANES")
        if env:
            return max(Rp, int(env))
        if self.ff.model_id == nat.MODEL_SR and self.ff.n_data() > 4:
            return Rp  # the wide-state kernel runs a workgroup per lane set already
        while Rp < 64 and (P + 64 // Rp - 1) // (64 // Rp) < self._simds():
            Rp *= 2
        return Rp

    def evaluate(self, pop: torch.Tensor, data, trajectories: bool = False, rollout_fitness: bool = False,
                 flattened: Optional[Flattened] = None, check: bool = True, schedule: bool = True,
                 step_counts: bool = False) -> dict:
        """Run flatten + fused RK4 kernel.  Returns device tensors:
        fitness [P] (+ rollout_fitness [P, R], xs/ys/us/acts indexed [S, c, P*R]).
        The trajectory tensors are indexed [S, c, P*R] for every solver, but only a fixed-step
        solve stores them that way (contiguous, time-major rows); an adaptive solve writes
        lane-major rows [P*R, S, c] (ABI v20) and returns a permuted, NON-contiguous view of that
        buffer.  res["_traj_layout"] names the storage (nat.TRAJ_TIME_MAJOR / TRAJ_LANE_MAJOR):
        read the tensors through indexing or to_reference_layout, and never hand their
        data_ptr() to native code without checking it.
        schedule: pair expensive with cheap individuals in each wave (results are identical)."""
        d = self.prepare_data(data)
        fl = flattened if flattened is not None else self.flatten(pop)
        P = pop.shape[0]
        R, S = d["R"], d["n_save"]
        m = self.model_struct(d)
        ro = self.rollouts_struct(d, P)
        lanes = ro.lanes
        ro_order = self.schedule(fl, lanes) if schedule and P > 1 else None
        ro.order = _ptr(ro_order)
        dev = self.device
        res = {"fitness": torch.empty((P,), dtype=torch.float32, device=dev)}
        out = nat.MtgpOutputs()
        out.fitness = res["fitness"].data_ptr()
        if rollout_fitness or lanes > 64:  # R > 64: the fitness mean is formed from it (mtgp.h)
            rf = torch.empty((P, R), dtype=torch.float32, device=dev)
            if rollout_fitness:
                res["rollout_fitness"] = rf
            else:
                res["_rollout_fitness"] = rf
            out.rollout_fitness = rf.data_ptr()
        if step_counts:  # Dopri5: step attempts per (individual, rollout)
            res["steps"] = torch.zeros((P, R), dtype=torch.int32, device=dev)
            out.steps = res["steps"].data_ptr()
        # Dopri5 in two launches: the waves still integrating after max_steps / 2 attempts are parked
        # and resumed by a second launch that spreads them over all SIMDs (DESIGN.md "Dopri5 tail":
        # C3 + obs_noise 0.1, the notebooks' setting, 70.6 -> 58.4 ms; without noise 31.2 vs 32.1)
        # (state_size > 3: one launch -- the runtime-state-size Dopri5 kernel does not park)
        dp_ctl = m.solver == nat.SOLVER_DOPRI5 and self.ff.model_id != nat.MODEL_SR and m.state_size <= 3
        budget = self.dp_budget if self.dp_budget is not None else (self._dp_choose(m.max_steps) if dp_ctl else 0)
        if dp_ctl and budget > 0:
            waves = self.native.mtgp_eval_waves(P, R, lanes)
            if waves < 0:
                raise RuntimeError(f"mtgp_eval_waves({P}, {R}, {lanes}) failed")
            if self._dp_bufs is None or self._dp_bufs[0].numel() < nat.DP_STATE_WORDS * waves * 64:
                self._dp_bufs = (torch.empty((nat.DP_STATE_WORDS * waves * 64,), dtype=torch.float32, device=dev),
                                 torch.empty((1 + waves,), dtype=torch.int32, device=dev))
            m.dp_budget = budget
            out.dp_state, out.dp_pending = self._dp_bufs[0].data_ptr(), self._dp_bufs[1].data_ptr()
        if d.get("fit_need_hist"):  # the general Acrobot mask's cost prefixes (mtgp.h fit_hist)
            res["_fit_hist"] = torch.empty((S * P * R,), dtype=torch.float32, device=dev)
            out.fit_hist = res["_fit_hist"].data_ptr()
        if trajectories:
            PR = P * R
            # Adaptive solves write lane-major rows (mtgp.h traj_layout, ABI v20: each lane's divergent
            # save points land contiguously -- half the write traffic); the result is handed back as
            # the same [S, c, P*R] tensor a fixed-step solve gives, a strided view of the [P*R, S, c]
            # buffer (whose [P, R, S, c] reading is the reference's layout: to_reference_layout).
            # MTGP_TRAJ_LAYOUT=time forces time-major rows (A/B).
            lane_major = m.solver == nat.SOLVER_DOPRI5 and os.environ.get("MTGP_TRAJ_LAYOUT", "auto") != "time"
            out.traj_layout = nat.TRAJ_LANE_MAJOR if lane_major else nat.TRAJ_TIME_MAJOR
            res["_traj_layout"] = out.traj_layout
            names = (("xs", m.n_var),) if self.ff.model_id == nat.MODEL_SR else \
                (("xs", m.n_var), ("ys", m.n_obs), ("us", m.n_control), ("acts", m.state_size))
            for name, c in names:
                if c > 0:
                    if lane_major:
                        buf = torch.empty((PR, S, c), dtype=torch.float32, device=dev)
                        res[name] = buf.permute(1, 2, 0)
                    else:
                        buf = res[name] = torch.empty((S, c, PR), dtype=torch.float32, device=dev)
                    setattr(out, name, buf.data_ptr())
        stream = torch.cuda.current_stream(dev).cuda_stream
        jit = self.jit_build(fl, m, lanes, ro_order)
        jc = nat.MtgpJitCode()
        if jit is not None:
            jc.code, jc.offsets, jc.info, jc.capacity = jit[0], jit[1].data_ptr(), jit[2].data_ptr(), jit[3]
            jc.chain = jit[4]
        rc = self.native.mtgp_eval_rk4_jit(ctypes.byref(m), fl.prog.data_ptr(), fl.plen.data_ptr(), fl.n_prog, fl.L,
                                           fl.nodes.data_ptr(), P, ctypes.byref(ro), ctypes.byref(out),
                                           ctypes.byref(jc), stream)
        if rc != nat.OK:
            raise RuntimeError(f"mtgp_eval_rk4 rejected the configuration (code {rc})")
        if dp_ctl and budget > 0 and self.dp_budget is None and self._dp_probe is None:
            # the parked-wave count, read back lazily (one pinned word, reused once consumed)
            if self._dp_pinned is None:
                self._dp_pinned = torch.empty((1,), dtype=torch.int32, pin_memory=True)
            self._dp_pinned.copy_(self._dp_bufs[1][:1], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(dev))
            self._dp_probe = (ev, self._dp_pinned, waves)
        if check:
            self.check_status(fl)
        res["_flat"] = fl
        return res

    # Two launches pay when many waves are still integrating after max_steps / 2 attempts (launch 2
    # spreads them over the SIMDs) and cost when few are: measured on the C3 Dopri5 workload with
    # lane-major rows (profiles/r05/v27_dpab_*.log), noise-free 288 of 4,096 waves parked, one launch
    # 18.2 ms vs two 20.1 ms; obs_noise 0.1 1,587 parked, one launch 64.5 ms vs two 55.1 ms.  So the
    # automatic budget is one launch while the last two-launch evaluation parked fewer than
    # kDpOneLaunchFrac of its waves, re-probed with two launches every kDpProbeEvery evaluations
    # (populations drift over generations).  Results are bit-identical for every budget.
    kDpOneLaunchFrac = 0.2
    kDpProbeEvery = 16

    def _dp_choose(self, max_steps: int) -> int:
        self._dp_evals += 1
        if self._dp_probe is not None:
            ev, cnt, waves = self._dp_probe
            if ev.query():
                self._dp_frac = int(cnt[0]) / max(waves, 1)
                self._dp_probe = None
        two = max_steps // 2
        if self._dp_frac is None or self._dp_evals % self.kDpProbeEvery == 0:
            return two
        return 0 if self._dp_frac < self.kDpOneLaunchFrac else two

    def eval_programs(self, fl: Flattened, data_vectors: torch.Tensor) -> torch.Tensor:
        """Batched tree_evaluator: every program on M data vectors -> [P, n_prog, M]."""
        P = fl.prog.shape[0]
        M, D = data_vectors.shape
        out = torch.empty((P, fl.n_prog, M), dtype=torch.float32, device=self.device)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        rc = self.native.mtgp_eval_programs(fl.prog.data_ptr(), fl.plen.data_ptr(), fl.n_prog, fl.L, P,
                                            data_vectors.data_ptr(), M, D, out.data_ptr(), stream)
        if rc != nat.OK:
            raise RuntimeError(f"mtgp_eval_programs failed: {rc}")
        return out


def to_reference_layout(t: torch.Tensor, P: int, R: int) -> np.ndarray:
    """time-major [S, c, P*R] -> evaluate_candidate layout [P, R, S, c] (host numpy)."""
    S, c, _ = t.shape
    return t.reshape(S, c, P, R).permute(2, 3, 0, 1).contiguous().cpu().numpy()
