#!/usr/bin/env python3
"""One library's fixed-length kernel at the given lengths (KVH_LIB selects
the build; one process per library): HIP-event medians over 100M keys, and
a checksum of the output so builds can be compared.  Usage:
KVH_LIB=... python tools/len_ab.py TAG L [L ...]"""
import json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raikv_amd as kvh  # noqa: E402

torch.cuda.set_device(0)
tag, lens = sys.argv[1], [int(x) for x in sys.argv[2:]]
st = torch.cuda.current_stream()
n = 100_000_000
out = torch.empty((n, 2), dtype=torch.int64, device="cuda")
for L in lens:
    g = torch.Generator(device="cuda").manual_seed(L)
    keys = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    kvh.meow128_fixed(keys, L, kvh.STATIC_SEED, out=out)
    torch.cuda.synchronize()
    chk = int(out.view(torch.int64).sum().item()) & 0xFFFFFFFFFFFFFFFF
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
    for a, b in ev:
        a.record(st); kvh.meow128_fixed(keys, L, kvh.STATIC_SEED, out=out); b.record(st)
    torch.cuda.synchronize()
    t = float(np.median([a.elapsed_time(b) for a, b in ev]))
    print(json.dumps({"lib": tag, "L": L, "median_ms": round(t, 4), "Gkeys_s": round(n / t / 1e6, 2),
                      "checksum": hex(chk)}), flush=True)
    del keys
