#!/usr/bin/env python3
"""A/B of the table-order sort (kvh_set_tuning(17, bits): h1 bits sorted
below the slot bits; 64 = the full 64-bit key; or, with TUNE_KNOB=20, the
engines: 0 two-pass bucketed, 2 one-pass bucketed, 1 radix) on bench.py's
f2 workload; outputs asserted equal."""
import json, os, sys
KNOB = int(os.environ.get("TUNE_KNOB", "17"))
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raikv_amd as kvh  # noqa: E402

torch.cuda.set_device(0)
n = 100_000_000
g = torch.Generator(device="cuda"); g.manual_seed(1)
keys = torch.randint(0, 256, (n * 16,), dtype=torch.uint8, device="cuda", generator=g)
h = kvh.meow128_fixed(keys, 16, kvh.STATIC_SEED, fixup=True)
del keys
nd = n // 100
h[torch.randperm(n, device="cuda", generator=g)[:nd]] = h[torch.randint(0, n, (nd,), device="cuda", generator=g)]
items = torch.arange(n, dtype=torch.int64, device="cuda")
geom = kvh.HtGeom.from_map(64 << 30, 64, 1.0, 4, 4)
srt = kvh.HtSorter(geom, n)
ho, io = torch.empty_like(h), torch.empty_like(items)
ref = None
res = {}
st = torch.cuda.current_stream()
for r in range(3):
    for bits in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "64,16,8").split(",")]:
        kvh.lib.kvh_set_tuning(KNOB, bits)
        srt.sort(h, items, dedup=True, out=ho, items_out=io)
        torch.cuda.synchronize()
        if ref is None: ref = (ho.clone(), io.clone(), int(srt.dups.item()))
        elif not (KNOB == 23 and (7 <= bits <= 10 or 12 <= bits <= 15)):  # knob 23 = 7-10, 12-15: phase ablations, outputs not sorted
            assert torch.equal(ho, ref[0]) and torch.equal(io, ref[1]) and int(srt.dups.item()) == ref[2], bits
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(3)]
        for a, b in ev:
            a.record(st); srt.sort(h, items, dedup=True, out=ho, items_out=io); b.record(st)
        torch.cuda.synchronize()
        res.setdefault(bits, []).extend(a.elapsed_time(b) for a, b in ev)
kvh.lib.kvh_set_tuning(KNOB, {20: 0, 23: 3}.get(KNOB, 16))
for bits, t in res.items():
    ms = float(np.median(t))
    print(json.dumps({"knob": KNOB, "value": bits, "median_ms": ms, "Gkeys_s": n / ms / 1e6, "dups": ref[2]}))
