#!/usr/bin/env python3
"""A/B of the span-hash kernels (kvh_set_tuning(18, v): 2 / 1 two / one spans
per lane with the short-key path and medium/long queues, 0 lane per span;
3 and 4 ablations: no table rounds; offsets/lengths in and hashes out only)
on bench.py's f3 text (1 GiB, ~25 % separators, ~200M tokens); outputs of
the product kernels asserted equal."""
import json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raikv_amd as kvh  # noqa: E402

torch.cuda.set_device(0)
n = 1 << 30
g = torch.Generator(device="cuda"); g.manual_seed(1000)
r = torch.randint(0, 8, (n,), dtype=torch.uint8, device="cuda", generator=g)
text = torch.where(r == 0, 32, torch.where(r == 1, 10, 97 + r)).to(torch.uint8)
del r
offs, lens = kvh.tokenize(text, 256)
k = offs.numel()
out = torch.empty((k, 2), dtype=torch.int64, device="cuda")
st = torch.cuda.current_stream()
ref, res = None, {v: [] for v in (0, 1, 2, 3, 4)}
for rnd in range(3):
    for v in (0, 1, 2, 3, 4):
        kvh.lib.kvh_set_tuning(18, v)
        kvh.meow128_spans(text, offs, lens, kvh.STATIC_SEED, out=out)
        torch.cuda.synchronize()
        if ref is None: ref = out.clone()
        elif v < 3: assert torch.equal(ref, out), v  # 3, 4: ablations (not hashes)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
        for a, b in ev:
            a.record(st); kvh.meow128_spans(text, offs, lens, kvh.STATIC_SEED, out=out); b.record(st)
        torch.cuda.synchronize()
        res[v] += [a.elapsed_time(b) for a, b in ev]
kvh.lib.kvh_set_tuning(18, 1)
for v, t in res.items():
    ms = float(np.median(t))
    print(json.dumps({"spans_kernel": v, "tokens": k, "median_ms": ms, "Gtok_s": k / ms / 1e6}))
