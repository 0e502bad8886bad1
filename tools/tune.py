#!/usr/bin/env python3
"""A/B the fixed-length kernel variants in ONE process, interleaved rounds
(guide §5.4 rule 24).  Prints per-variant median/min kernel ms and GB/s."""
import os as _os  # research knobs live in the experiments build (make experiments)
_os.environ.setdefault("KVH_LIB", _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "libkvh_exp.so"))
import argparse
import itertools
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raikv_amd as kvh  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=100_000_000)
ap.add_argument("--L", type=int, default=16)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--variants", default="nt=4,2;kpl=1,2;wg=1")
ap.add_argument("--arity", type=int, default=1)
a = ap.parse_args()

torch.cuda.set_device(0)
g = torch.Generator(device="cuda")
g.manual_seed(5)
keys = torch.randint(0, 256, (a.n * a.L,), dtype=torch.uint8, device="cuda", generator=g)
out = torch.empty((a.n, a.arity, 2), dtype=torch.int64, device="cuda")
seeds = [(1, 2), (3, 4), (5, 6), (7, 8)][: a.arity]
spec = dict(kv.split("=") for kv in a.variants.split(";"))
axes = {k: [int(x) for x in v.split(",")] for k, v in spec.items()}
knob = {"nt": 0, "wg": 1, "generic": 2, "kpl": 3, "dma": 6, "var": 7, "mslanes": 8, "pf": 10, "bs": 11, "bsw": 12, "prio": 13}
names = list(axes)
variants = list(itertools.product(*[axes[k] for k in names]))
ref = None
res = {v: [] for v in variants}
st = torch.cuda.current_stream()
for r in range(a.rounds):
    for v in variants:
        for k, val in zip(names, v):
            kvh.lib.kvh_set_tuning(knob[k], val)
        if a.arity == 1:
            f = lambda: kvh.meow128_fixed(keys, a.L, kvh.STATIC_SEED, out=out.view(a.n, 2))
        else:
            f = lambda: kvh.meow128_multiseed(keys, a.L, seeds, out=out)
        f()
        torch.cuda.synchronize()
        if ref is None:
            ref = out.clone()
        else:
            assert torch.equal(out, ref), f"variant {v} output differs"
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
        for e0, e1 in evs:
            e0.record(st); f(); e1.record(st)
        torch.cuda.synchronize()
        res[v] += [e0.elapsed_time(e1) for e0, e1 in evs]
byt = a.n * (a.L + 16 * a.arity)
rows = []
for v in variants:
    t = np.array(res[v])
    rows.append({"variant": dict(zip(names, v)), "median_ms": float(np.median(t)), "min_ms": float(t.min()),
                 "GBps_median": byt / np.median(t) / 1e6, "Ghash_s": a.n * a.arity / np.median(t) / 1e6})
for r in sorted(rows, key=lambda r: r["median_ms"]):
    print(json.dumps(r))
