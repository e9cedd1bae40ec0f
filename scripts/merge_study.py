#!/usr/bin/env python3
"""Design study (CPU): how much of C5's program work could a lane-merged unit save?

A C5 wave holds G = 8 individuals x 8 rollouts; unit (wave, component j) runs the 8 groups'
programs one after another with full exec, so every lane executes 8 programs to keep one.  A
merged unit would run ONE instruction stream in which each position is an operation every lane
applies to its own operands (the operand stack depth resolved per position, data slots and
constants fetched per lane).  The stream is a common supersequence of the 8 token sequences
(token = opcode + stack depth); this reports, over the bench population, the ratio of the
greedy (majority-merge) supersequence length to the summed program lengths, plain and weighted
by the JIT's executed words per opcode.

    python scripts/merge_study.py --waves 32"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from multitreegp_amd import _native as nat  # noqa: E402

PUSH = {"LDCP", "LDVP", "SINVP", "COSVP"}


def tokens(prog):
    sp, out = 0, []
    for ins in prog:
        name = ins[0]
        out.append((name, sp))
        if name in PUSH or name.startswith("VCP_") or name.startswith("VVP_"):
            sp += 1
        elif name in ("ADDS", "SUBS", "RSUBS", "MULS", "DIVS", "RDIVS"):
            sp -= 1
    return out


def weight(name):
    if "DIV" in name:
        return 12.0
    if "SIN" in name or "COS" in name:
        return 40.0
    return 1.0


def majority_merge(seqs, w):
    pos = [0] * len(seqs)
    total = 0.0
    n = 0
    while True:
        live = [i for i, s in enumerate(seqs) if pos[i] < len(s)]
        if not live:
            return n, total
        votes = collections.Counter()
        for i in live:
            t = seqs[i][pos[i]]
            votes[t] += len(seqs[i]) - pos[i]  # favour sequences with more left
        t = votes.most_common(1)[0][0]
        for i in live:
            if seqs[i][pos[i]] == t:
                pos[i] += 1
        n += 1
        total += w(t[0])


ap = argparse.ArgumentParser()
ap.add_argument("--waves", type=int, default=32)
ap.add_argument("--G", type=int, default=8)
a = ap.parse_args()
args = argparse.Namespace(pop=a.waves * a.G, rollouts=8, ode_steps=200, config="c5")
env, lib, ff, data, P = bench.setup_workload(args, 0)
ff.prepare(data)
specs, _ = ff.program_specs()
nl = lib.native()
tot_n = tot_w = m_n = m_w = 0.0
for wv in range(a.waves):
    for t, d, z in specs:
        seqs = []
        for g in range(a.G):
            prog, _ = nat.flatten_tree_host(P[wv * a.G + g, t], nl, d, z)
            seqs.append(tokens(prog))
        tot_n += sum(len(s) for s in seqs)
        tot_w += sum(weight(x[0]) for s in seqs for x in s)
        n, wsum = majority_merge(seqs, weight)
        m_n += n
        m_w += wsum
print(f"instructions: separate {tot_n:.0f}, merged {m_n:.0f}, ratio {m_n / tot_n:.3f}")
print(f"weighted:     separate {tot_w:.0f}, merged {m_w:.0f}, ratio {m_w / tot_w:.3f}")
