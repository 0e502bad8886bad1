#!/usr/bin/env python3
"""A/B of the fixed-length chunk order (kvh_set_tuning(24, v): 0 = static
per-wave order, k_fixed; 1/2/3 = in address order from a ticket counter,
k_fixed_q with 1/4/16 workgroup-rounds per ticket) on the C1 / C4 / C64 shapes, one process, interleaved
rounds after a 500 ms settle, outputs asserted equal.  One JSON line per
(shape, order)."""
import json, os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raikv_amd as kvh  # noqa: E402

torch.cuda.set_device(0)
shapes = [(16, 100_000_000), (32, 125_000_000), (64, 100_000_000)]
if len(sys.argv) > 1:
    shapes = [s for s in shapes if str(s[0]) in sys.argv[1].split(",")]
st = torch.cuda.current_stream()
VS = [int(x) for x in os.environ.get("ORDERS", "0,1,2,3").split(",")]
g = torch.Generator(device="cuda")
g.manual_seed(7)
for L, n in shapes:
    keys = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    out = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    ref = None
    for v in VS:
        kvh.lib.kvh_set_tuning(24, v)
        kvh.meow128_fixed(keys, L, kvh.STATIC_SEED, out=out)
        torch.cuda.synchronize()
        if ref is None:
            ref = out.clone()
        else:
            assert torch.equal(ref, out), f"order {v} differs at L={L}"
    del ref
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        kvh.meow128_fixed(keys, L, kvh.STATIC_SEED, out=out)
        torch.cuda.synchronize()
    res = {v: [] for v in VS}
    for r in range(6):
        for v in VS:
            kvh.lib.kvh_set_tuning(24, v)
            kvh.meow128_fixed(keys, L, kvh.STATIC_SEED, out=out)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
            for a, b in ev:
                a.record(st)
                kvh.meow128_fixed(keys, L, kvh.STATIC_SEED, out=out)
                b.record(st)
            torch.cuda.synchronize()
            res[v] += [a.elapsed_time(b) for a, b in ev]
    kvh.lib.kvh_set_tuning(24, 0)
    for v in VS:
        ms = float(np.median(res[v]))
        print(json.dumps({"key_len": L, "n": n, "order": ["static", "tickets_r1", "tickets_r4", "tickets_r16", "wave_tickets"][v],
                          "median_ms": ms,
                          "min_ms": float(np.min(res[v])), "G_hash_s": n / ms / 1e6,
                          "alg_TBps": n * (L + 16) / ms / 1e9}), flush=True)
    del keys, out
    torch.cuda.empty_cache()
