#!/usr/bin/env python3
"""Fixed-length throughput across key lengths 8..64 (the BASELINE metric's
16-64 B range and its neighbours): kvh_meow128_fixed on 50M keys per
length, median of 5 timed launches, product library.  One JSON line per
length; outputs spot-checked against the variable-length kernel."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raikv_amd as kvh  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000_000
lens = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else list(range(8, 65, 4)) + [15, 17, 31, 33, 63]
torch.cuda.set_device(0)
g = torch.Generator(device="cuda")
g.manual_seed(1)
keys = torch.randint(0, 256, (n * 64,), dtype=torch.uint8, device="cuda", generator=g)
out = torch.empty((n, 2), dtype=torch.int64, device="cuda")
st = torch.cuda.current_stream()
for L in sorted(lens):
    kb = keys[: n * L]
    kvh.meow128_fixed(kb, L, kvh.STATIC_SEED, out=out)
    # spot check: 4096 keys through the variable-length path
    m = 4096
    offs = torch.arange(0, (m + 1) * L, L, dtype=torch.int64, device="cuda")
    ref = kvh.meow128_var(kb[: m * L], offs, kvh.STATIC_SEED)
    assert torch.equal(ref, out[:m]), L
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        kvh.meow128_fixed(kb, L, kvh.STATIC_SEED, out=out)
        e1.record(st)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    t = float(np.median(ts))
    print(json.dumps({"key_len": L, "n": n, "ms": round(t, 3), "Ghash_s": round(n / t / 1e6, 1),
                      "alg_TBps": round(n * (L + 16) / t / 1e9, 2)}), flush=True)
