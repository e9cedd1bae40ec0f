#!/usr/bin/env python3
"""Dispatch frequencies (% of interpreted instructions, END included) of the flattened programs
of the bench workloads -- the weights of scripts/gen_opcodes.py's Huffman dispatch tree."""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from multitreegp_amd import _native as nat  # noqa: E402


def freqs(config, pop, stride):
    a = argparse.Namespace(pop=pop, rollouts=8, ode_steps=200, config=config)
    env, lib, ff, data, P = bench.setup_workload(a, 0)
    ff.prepare(data)
    specs, _ = ff.program_specs()
    nl = lib.native()
    c = collections.Counter()
    for p in range(0, P.shape[0], stride):
        for t, d, z in specs:
            prog, _ = nat.flatten_tree_host(P[p, t], nl, d, z)
            c.update(x[0] for x in prog)
            c["END"] += 1
    n = sum(c.values())
    return {k: round(100.0 * v / n, 2) for k, v in c.most_common()}, n


if __name__ == "__main__":
    for cfg, pop, stride in (("c3", 2048, 4), ("c5", 64, 1)):
        f, n = freqs(cfg, pop, stride)
        print(f"# {cfg}: {n} dispatches")
        print(f"FREQ_{'C3' if cfg == 'c3' else 'SR'} = {f!r}")
