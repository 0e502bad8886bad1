#!/usr/bin/env python3
"""Ablation of k_var3 (KPT=4) on config C2: product / no-hash / no-gather / no-sort."""
import os as _os  # research knobs live in the experiments build (make experiments)
_os.environ.setdefault("KVH_LIB", _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "libkvh_exp.so"))
import json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raikv_amd as kvh  # noqa: E402
from raikv_amd.workload import zipf_lengths, offsets_from_lengths  # noqa: E402
torch.cuda.set_device(0)
n = 100_000_000
offs = offsets_from_lengths(zipf_lengths(n, 8, 256, seed=3))
keys = torch.randint(0, 256, (int(offs[-1]),), dtype=torch.uint8, device="cuda")
doff = torch.from_numpy(offs.view(np.int64)).cuda()
out = torch.empty((n, 2), dtype=torch.int64, device="cuda")
kvh.lib.kvh_set_tuning(7, 5)
res = {m: [] for m in range(4)}
st = torch.cuda.current_stream()
for r in range(3):
    for m in range(4):
        kvh.lib.kvh_set_tuning(9, m)
        kvh.meow128_var(keys, doff, kvh.STATIC_SEED, out=out)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(3)]
        for a, b in ev:
            a.record(st); kvh.meow128_var(keys, doff, kvh.STATIC_SEED, out=out); b.record(st)
        torch.cuda.synchronize()
        res[m] += [a.elapsed_time(b) for a, b in ev]
names = {0: "product", 1: "no-hash (sort+gather+store)", 2: "no-gather (sort+hash+store)", 3: "no-sort (gather+hash+store)"}
for m in range(4):
    t = float(np.median(res[m]))
    print(json.dumps({"mode": names[m], "median_ms": t, "Gkeys_s": n / t / 1e6}))
