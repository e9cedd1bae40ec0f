"""The per-population build chain on the GPU: mtgp_flatten_ex (LDS-staged flatten + JIT sizing)
and the word-based JIT plan / emit must reproduce the host flattener and the translation-based
mtgp_jit_plan / mtgp_jit_emit exactly (programs, lengths, status, node counts, unit offsets, plan
status and every code byte)."""
import ctypes

import numpy as np
import pytest

import multitreegp_amd as mt
from multitreegp_amd import _native as nat
from multitreegp_amd.sampling import sample_population

from helpers import CONTROL_OPS, SR_OPS, bits_equal, mismatch_report, tree_from_expr

pytestmark = pytest.mark.gpu


def _flatten_ex(pop, lib, specs, L, mode=0):
    import torch
    P, T, N, _ = pop.shape
    L_ = nat.load()
    dev = torch.device("cuda", 0)
    n_prog = len(specs)
    arr = (nat.MtgpProgramSpec * n_prog)()
    for i, (t, d, z) in enumerate(s[:3] for s in specs):
        arr[i].tree, arr[i].n_data, arr[i].zero_mask = t, d, z
    sp = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(dev)
    pd = torch.from_numpy(np.ascontiguousarray(pop, np.float32)).to(dev)
    prog = torch.empty((P * n_prog * L * 2 + 8,), dtype=torch.int32, device=dev)
    out = {k: torch.empty(s, dtype=torch.int32, device=dev) for k, s in
           (("plen", (P, n_prog)), ("nodes", (P,)), ("status", (P, n_prog)), ("jw", (P, n_prog)), ("jc", (P, n_prog)))}
    libs = lib.native()
    rc = L_.mtgp_flatten_ex(pd.data_ptr(), P, T, N, ctypes.byref(libs), sp.data_ptr(), n_prog, L, prog.data_ptr(),
                            out["plen"].data_ptr(), out["nodes"].data_ptr(), out["status"].data_ptr(),
                            out["jw"].data_ptr(), out["jc"].data_ptr(), mode, None)
    assert rc == nat.OK
    torch.cuda.synchronize()
    return prog, out


def _population(kind, P, seed=0):
    rng = np.random.default_rng(seed)
    if kind in ("dynamic", "dynamic3"):
        vl = [["y1", "y2", "y3", "y4", "a1", "a2", "u"], ["a1", "a2"]]
        lib = mt.NodeLibrary(CONTROL_OPS, vl, [2, 1])
        pop = sample_population(seed, lib, P, 1, max_init_depth=10, max_nodes=64)[0]
        specs = [(0, 7, 0), (1, 7, 0), (2, 7, 0b1001111), (2, 7, 0b1000000)]
        if kind == "dynamic3":  # an odd number of programs (two per flatten wave: the last half idle)
            specs = specs[:3]
    elif kind == "sr40":  # 40 variables, deep trees: programs read more than kJitPreSlots distinct slots
        lib = mt.NodeLibrary(SR_OPS, [[f"x{i}" for i in range(40)]], [4])
        pop = sample_population(seed, lib, P, 1, max_init_depth=9, max_nodes=128)[0]
        specs = [(i, 40, 0) for i in range(4)]
        # the sampler's trees are small (operator probability 0.7^depth, initialization.py:35):
        # every 7th individual gets balanced trees over 17-40 distinct variables
        ops = ["+", "-", "*", "/"]

        def balanced(vs, k=0):
            if len(vs) == 1:
                return vs[0]
            h = len(vs) // 2
            return (ops[k % 4], balanced(vs[:h], k + 1), balanced(vs[h:], k + 2))

        for p in range(0, P, 7):
            for t in range(4):
                m = int(rng.integers(17, 41))
                vs = [f"x{int(i)}" for i in rng.permutation(40)[:m]]
                pop[p, t] = tree_from_expr(balanced(vs), lib, 128)
    else:  # 12-variable SR: slots >= 8 are untranslatable -> negative jit words
        lib = mt.NodeLibrary(SR_OPS, [[f"x{i}" for i in range(12)]], [12])
        pop = sample_population(seed, lib, P, 1, max_init_depth=6, max_nodes=40)[0]
        specs = [(i, 12, 0) for i in range(12)]
    g = rng.random(pop.shape[:1]) < 0.1  # garbage individuals: arbitrary arrays
    junk = rng.normal(0, 8, size=pop.shape).astype(np.float32)
    pop[g] = junk[g]
    return lib, pop, specs


@pytest.mark.parametrize("halves", ["1", "0"])
@pytest.mark.parametrize("kind,mode", [("dynamic", 0), ("dynamic3", 0), ("sr12", 0), ("sr12", 1), ("sr40", 1),
                                       ("dynamic", 1)])
def test_flatten_ex_matches_host_flatten_and_jit_sizes(kind, mode, halves, monkeypatch):
    """MTGP_FLAT_HALVES=1 forces two programs per flatten wave (trees of <= 64 rows, register-mode
    sizing; by default only launches of more than 8,192 programs pack), 0 one per wave."""
    monkeypatch.setenv("MTGP_FLAT_HALVES", halves)
    lib, pop, specs = _population(kind, 301)
    P, T, N, _ = pop.shape
    L = (2 * N + 8 + 3) // 4 * 4
    prog, out = _flatten_ex(pop, lib, specs, L, mode)
    progs = prog[: P * len(specs) * L * 2].view(P, len(specs), L, 2).cpu().numpy()
    plen, status, jw, jc = (out[k].cpu().numpy() for k in ("plen", "status", "jw", "jc"))
    nodes = out["nodes"].cpu().numpy()
    L_ = nat.load()
    libs = lib.native()
    host = np.zeros((L, 2), np.int32)
    word = np.zeros(4096, np.uint32)
    for p in range(P):
        assert nodes[p] == int((pop[p, ..., 0] != 0).sum())
        for j, (t, d, z) in enumerate(s[:3] for s in specs):
            n = L_.mtgp_flatten_tree_host(pop[p, t].ctypes.data, N, ctypes.byref(libs), d, z, L, host.ctypes.data,
                                          None)
            assert plen[p, j] == max(n, 0) and status[p, j] == (0 if n > 0 else -n), (p, j)
            assert np.array_equal(progs[p, j, : max(n, 0) + 1], host[: max(n, 0) + 1]), (p, j)
            w = L_.mtgp_jit_translate_host_ex(host.ctypes.data, L, word.ctypes.data, 4096, mode)
            assert jw[p, j] == (w - 1 if w > 0 else w + 100), (p, j, jw[p, j], w)
    import torch
    cost = torch.empty((P, len(specs)), dtype=torch.int32, device="cuda")
    if mode == 0:
        assert L_.mtgp_jit_cost(prog.data_ptr(), out["plen"].data_ptr(), P, len(specs), L, cost.data_ptr(), None) == 0
        assert np.array_equal(cost.cpu().numpy(), jc)
    if kind == "sr12":
        assert ((jw < 0).any() if mode == 0 else (jw >= 0).all()) and (jw > 0).any()
    if kind == "sr40":  # some programs load slots at their use (more than 16 distinct slots)
        sb = nat.SLOT_BYTES
        distinct = [len({int(w) // sb for w in progs[p, j, :plen[p, j], 1].view(np.uint32) if w < 40 * sb})
                    for p in range(P) for j in range(len(specs)) if status[p, j] == 0]
        assert max(distinct) > 16


@pytest.mark.parametrize("emit", ["quarters", "halves", "wave64"])
@pytest.mark.parametrize("kind", ["dynamic", "sr12"])
@pytest.mark.parametrize("R", [1, 8, 32, 64])
def test_word_based_jit_plan_and_emit_match_translation(kind, R, emit, monkeypatch):
    """Register-mode units from the word-based plan and emit equal the thread-per-unit translation:
    the default emitter (four (unit, group) pairs per wave, 16 lanes each), two per wave
    (MTGP_JIT_EMIT=halves) and one wave per pair (MTGP_JIT_EMIT=wave64)."""
    import torch
    monkeypatch.setenv("MTGP_JIT_EMIT", emit)  # (by default the packing follows the launch size)
    lib, pop, specs = _population(kind, 257, seed=R)
    P, T, N, _ = pop.shape
    n_prog = len(specs)
    L = (2 * N + 8 + 3) // 4 * 4
    prog, out = _flatten_ex(pop, lib, specs, L)
    L_ = nat.load()
    order = torch.from_numpy(np.random.default_rng(R).permutation(P).astype(np.int32)).cuda()
    n = L_.mtgp_jit_units(P, n_prog, R)
    offs = [torch.empty((n + 1,), dtype=torch.int32, device="cuda") for _ in range(2)]
    info = [torch.zeros((2,), dtype=torch.int32, device="cuda") for _ in range(2)]
    assert L_.mtgp_jit_plan(prog.data_ptr(), P, n_prog, L, R, order.data_ptr(), offs[0].data_ptr(),
                            info[0].data_ptr(), None) == 0
    assert L_.mtgp_jit_plan_words(out["jw"].data_ptr(), P, n_prog, R, order.data_ptr(), offs[1].data_ptr(),
                                  info[1].data_ptr(), None) == 0
    torch.cuda.synchronize()
    assert np.array_equal(offs[0].cpu().numpy(), offs[1].cpu().numpy())
    i0, i1 = info[0].cpu().numpy(), info[1].cpu().numpy()
    assert (i0[0] < 0) == (i1[0] < 0) and i0[1] == i1[1]
    if kind == "sr12":
        assert i1[0] < 0
        return
    size = int(i1[1]) + 4096
    # emit writes words only, so plain device buffers stand in for executable memory here
    bufs = [torch.zeros((size // 4,), dtype=torch.int32, device="cuda") for _ in range(2)]
    assert L_.mtgp_jit_emit(prog.data_ptr(), P, n_prog, L, R, order.data_ptr(), offs[0].data_ptr(),
                            bufs[0].data_ptr(), size, None) == 0
    assert L_.mtgp_jit_emit_words(prog.data_ptr(), out["jw"].data_ptr(), P, n_prog, L, R, order.data_ptr(),
                                  offs[1].data_ptr(), bufs[1].data_ptr(), size, 0, None) == 0
    torch.cuda.synchronize()
    assert torch.equal(bufs[0], bufs[1])
    assert int((bufs[1] != 0).sum()) > size // 16


@pytest.mark.parametrize("emit", ["groups", "wave"])
@pytest.mark.parametrize("kind", ["sr12", "sr40"])
@pytest.mark.parametrize("store", [0, 8])
@pytest.mark.parametrize("R", [8, 64])
def test_lds_mode_units_match_host_units(R, store, kind, emit, monkeypatch):
    """LDS-data mode (wide-state SR): the device-built units equal the host-built ones word for word,
    plain or as LDS store chains (ABI v14: groups of 8 units packed back to back, each group ending
    on a 64-byte line), from the default thread-per-group emitter and from the wave-per-group one
    (MTGP_JIT_EMIT=wave, round 4); sr40's programs read more than kJitPreSlots distinct slots (loads
    at the use) and run 264 rows."""
    import torch
    if emit == "wave":
        monkeypatch.setenv("MTGP_JIT_EMIT", "wave")
    lib, pop, specs = _population(kind, 129, seed=R)
    P, T, N, _ = pop.shape
    n_prog = len(specs)
    L = (2 * N + 8 + 3) // 4 * 4
    prog, out = _flatten_ex(pop, lib, specs, L, 1)
    L_ = nat.load()
    order_np = np.random.default_rng(R).permutation(P).astype(np.int32)
    order = torch.from_numpy(order_np).cuda()
    n = L_.mtgp_jit_units(P, n_prog, R)
    offs = torch.empty((n + 1,), dtype=torch.int32, device="cuda")
    info = torch.zeros((2,), dtype=torch.int32, device="cuda")
    ch = nat.MtgpJitChain(0, 0, store)
    assert L_.mtgp_jit_plan_words_chain(out["jw"].data_ptr(), P, n_prog, R, order.data_ptr(), ctypes.byref(ch),
                                        offs.data_ptr(), info.data_ptr(), None) == 0
    torch.cuda.synchronize()
    inf = info.cpu().numpy()
    assert inf[0] == 0
    size = int(inf[1]) + 4096
    buf = torch.zeros((size // 4,), dtype=torch.int32, device="cuda")
    assert L_.mtgp_jit_emit_words_chain(prog.data_ptr(), out["jw"].data_ptr(), P, n_prog, L, R, order.data_ptr(),
                                        ctypes.byref(ch), offs.data_ptr(), buf.data_ptr(), size, 1, None) == 0
    torch.cuda.synchronize()
    code = buf.cpu().numpy().view(np.uint32)
    o = offs.cpu().numpy().view(np.uint32)
    hp = prog[: P * n_prog * L * 2].cpu().numpy()
    host = np.zeros(1 << 16, np.uint32)
    for u in range(0, n, max(1, n // 97)):
        w = L_.mtgp_jit_unit_host_chain(hp.ctypes.data, P, n_prog, L, R, order_np.ctypes.data, ctypes.byref(ch), u,
                                        host.ctypes.data, host.size, 1)
        assert w > 0
        j = u % n_prog
        if store and (j + 1) % store != 0 and j + 1 < n_prog:
            assert o[u + 1] - o[u] == 4 * w, u  # the next unit of the group follows directly
        else:
            assert o[u + 1] % 64 == 0, u
        # the units are laid out after the templates exactly as the host lays them out (PC-relative
        # calls aside, which SR has none of): equal words
        assert np.array_equal(code[o[u] // 4: o[u] // 4 + w], host[:w]), u


@pytest.mark.parametrize("form", ["merged", "cond"])
@pytest.mark.parametrize("R", [4, 32])
def test_chained_units_match_host_units(R, form):
    """Role chains (ABI v13): the device plan packs a chain member's successor right behind it
    (no alignment padding), every other unit starts on a 64-byte line, and the emitted code equals
    the host-built chained units word for word (the PC-relative literal of each sin/cos call
    aside: the host lays every unit out at the first code byte)."""
    import torch
    vl = [["y1", "y2", "y3", "y4", "a1", "a2", "u"], ["a1", "a2"]]
    lib = mt.NodeLibrary(CONTROL_OPS, vl, [2, 1])
    pop = sample_population(R, lib, 203, 1, max_init_depth=10, max_nodes=64)[0]
    specs = [(2, 7, 0b1001111), (0, 7, 0), (1, 7, 0), (2, 7, 0b1000000)]  # readout | state | save readout
    P, T, N, _ = pop.shape
    n_prog = len(specs)
    L = (2 * N + 8 + 3) // 4 * 4
    prog, out = _flatten_ex(pop, lib, specs, L)
    L_ = nat.load()
    m = nat.MtgpModel()
    m.model, m.state_size, m.n_var, m.solver = nat.MODEL_ACROBOT_DYNAMIC, 2, 4, nat.SOLVER_RK4
    m.prog_state, m.prog_readout, m.prog_readout_save, m.readout_save_same = 1, 0, 3, -1
    ch = nat.MtgpJitChain()
    assert L_.mtgp_jit_chain(ctypes.byref(m), n_prog, ctypes.byref(ch)) == 0
    assert (ch.next, ch.put, ch.put_slot) == (0b011, 0b001, 6)  # ABI v18: readout -> u slot -> state chain
    if form == "cond":  # the ABI v13 form with the conditional save continuation (emitter test)
        ch.next, ch.cond, ch.put, ch.put_slot = 0b110, 0b100, 0, 0
    order_np = np.random.default_rng(R).permutation(P).astype(np.int32)
    order = torch.from_numpy(order_np).cuda()
    n = L_.mtgp_jit_units(P, n_prog, R)
    offs = torch.empty((n + 1,), dtype=torch.int32, device="cuda")
    info = torch.zeros((2,), dtype=torch.int32, device="cuda")
    assert L_.mtgp_jit_plan_words_chain(out["jw"].data_ptr(), P, n_prog, R, order.data_ptr(), ctypes.byref(ch),
                                        offs.data_ptr(), info.data_ptr(), None) == 0
    torch.cuda.synchronize()
    inf = info.cpu().numpy()
    assert inf[0] == 0
    size = int(inf[1]) + 4096
    buf = torch.zeros((size // 4,), dtype=torch.int32, device="cuda")
    assert L_.mtgp_jit_emit_words_chain(prog.data_ptr(), out["jw"].data_ptr(), P, n_prog, L, R, order.data_ptr(),
                                        ctypes.byref(ch), offs.data_ptr(), buf.data_ptr(), size, 0, None) == 0
    torch.cuda.synchronize()
    code = buf.cpu().numpy().view(np.uint32)
    o = offs.cpu().numpy().view(np.uint32)
    hp = prog[: P * n_prog * L * 2].cpu().numpy()
    host = np.zeros(1 << 16, np.uint32)
    for u in range(n):
        j = u % n_prog
        w = L_.mtgp_jit_unit_host_chain(hp.ctypes.data, P, n_prog, L, R, order_np.ctypes.data, ctypes.byref(ch), u,
                                        host.ctypes.data, host.size, 0)
        assert w > 0
        if ch.next >> j & 1:
            assert o[u + 1] - o[u] == 4 * w, u  # the successor follows directly
        else:  # every unit that is called starts on a 64-byte line, chain members follow directly
            assert o[u] % 64 == 0 or (j > 0 and ch.next >> (j - 1) & 1), u
            assert o[u + 1] % 64 == 0 and o[u + 1] - o[u] >= 4 * w, u
        got = code[o[u] // 4: o[u] // 4 + w]
        keep = np.ones(w, bool)
        keep[1:] = got[:-1] != 0x802CFF2C  # s_add_u32 s44, literal: the PC-relative call offset
        assert np.array_equal(got[keep], host[:w][keep]), u


def test_chained_and_unchained_evaluations_agree():
    """The same population evaluated with chained JIT code, one-call-per-program JIT code
    (MTGP_JIT_CHAIN=0) and the interpreter: bit-identical fitness and trajectories (RK4 dynamic
    policy, SR n_var 2 chain)."""
    import os
    import torch
    from multitreegp_amd.engine import DeviceEngine
    env = mt.Acrobot(0.0, 0.0)
    lib = mt.NodeLibrary(CONTROL_OPS, [["y1", "y2", "y3", "y4", "a1", "a2", "u"], ["a1", "a2"]], [2, 1])
    ff = mt.DynamicEvaluator(env, 2, 0.05, solver=mt.RK4())
    data = mt.control_data(env, 32, 0.05, None, seed=3, n_steps=60)
    pop = torch.from_numpy(sample_population(11, lib, 130, 1, max_init_depth=10, max_nodes=64)[0]).cuda()
    outs = []
    for chain, jit in (("1", True), ("0", True), ("1", False)):
        os.environ["MTGP_JIT_CHAIN"] = chain
        try:
            eng = DeviceEngine(ff, lib, 0.5, "cuda:0", jit=jit)
            r = eng.evaluate(pop, data, trajectories=True)
            if jit:
                assert DeviceEngine.jit_ok(r["_flat"])
                assert (r["_flat"].jit[4].next != 0) == (chain == "1")
            outs.append({k: r[k].cpu().numpy() for k in ("fitness", "xs", "us", "acts", "ys")})
        finally:
            os.environ.pop("MTGP_JIT_CHAIN", None)
    # bit-identical, NaN == NaN whatever its sign bit (the parity rule of tests/helpers.bits_equal:
    # the sign of a NaN made by inf - inf follows the compiler's choice of sub vs add-with-neg)
    for name, o in zip(("unchained", "interpreter"), outs[1:]):
        for k in o:
            assert bits_equal(o[k], outs[0][k]), mismatch_report(o[k], outs[0][k], f"{name} {k}")
