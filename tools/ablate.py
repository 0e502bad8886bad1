#!/usr/bin/env python3
"""Ablation of the fixed-length kernel (kvh_set_tuning(5, mode)): product,
copy-only, no-load, no-store; interleaved rounds in one process."""
import os as _os  # research knobs live in the experiments build (make experiments)
_os.environ.setdefault("KVH_LIB", _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "libkvh_exp.so"))
import json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raikv_amd as kvh  # noqa: E402

torch.cuda.set_device(0)
for L, n in ((16, 100_000_000), (32, 50_000_000)):
    keys = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda")
    out = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    kvh.lib.kvh_set_tuning(0, 2); kvh.lib.kvh_set_tuning(3, 1)
    res = {m: [] for m in range(4)}
    st = torch.cuda.current_stream()
    for r in range(5):
        for m in range(4):
            kvh.lib.kvh_set_tuning(5, m)
            kvh.meow128_fixed(keys, L, kvh.STATIC_SEED, out=out)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
            for a, b in ev:
                a.record(st); kvh.meow128_fixed(keys, L, kvh.STATIC_SEED, out=out); b.record(st)
            torch.cuda.synchronize()
            res[m] += [a.elapsed_time(b) for a, b in ev]
    kvh.lib.kvh_set_tuning(5, 0)
    names = {0: "product", 1: "copy-only", 2: "no-load (LDS+store)", 3: "no-store (LDS+load)"}
    for m in range(4):
        t = float(np.median(res[m]))
        print(json.dumps({"L": L, "mode": names[m], "median_ms": t, "Gkeys_s": n / t / 1e6,
                          "GBps_alg": n * (L + 16) / t / 1e6}))
