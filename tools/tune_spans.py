#!/usr/bin/env python3
"""A/B of the span-hash kernel variants (kvh_set_tuning(18, v)) on bench.py's
f3 text (1 GiB, ~25 % separators, ~200M tokens), outputs asserted equal:
2 the product (wave tickets, two spans per lane, the short-key path and
medium/long queues), 1 the static-order form, 0 lane per span; with the
experiments build (KVH_LIB=tools/libkvh_exp.so) 3 = 2 with the short path's
second text block loaded only where the span crosses a 16-byte boundary;
4 / 5 traffic ablations (outputs not hashes): the first text block only / no
text loads on the short path; 6 = 2 with each queued span's (offset, length)
parked in its own output slot at the short-hash store and read back there.

    python tools/tune_spans.py [arms, default 2,3] [--once]

--once: each arm launched 5 times, no timing (for rocprofv3 --pmc runs)."""
import json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raikv_amd as kvh  # noqa: E402

arms = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else "2,3").split(",")]
once = "--once" in sys.argv
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
ref, res = None, {v: [] for v in arms}
for rnd in range(1 if once else 3):
    for v in arms:
        assert kvh.lib.kvh_set_tuning(18, v) >= 0, v
        kvh.meow128_spans(text, offs, lens, kvh.STATIC_SEED, out=out)
        torch.cuda.synchronize()
        if ref is None: ref = out.clone()
        elif v not in (4, 5): assert torch.equal(ref, out), v  # 4, 5: traffic ablations (not hashes)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
        for a, b in ev:
            a.record(st); kvh.meow128_spans(text, offs, lens, kvh.STATIC_SEED, out=out); b.record(st)
        torch.cuda.synchronize()
        res[v] += [a.elapsed_time(b) for a, b in ev]
kvh.lib.kvh_set_tuning(18, 2)
for v, t in res.items():
    ms = float(np.median(t))
    print(json.dumps({"spans_kernel": v, "tokens": k, "median_ms": ms, "Gtok_s": k / ms / 1e6}))
