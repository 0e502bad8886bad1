#!/usr/bin/env python3
"""Tables (Td0..Td3 or Td0/Td1, knob 0) and keys per lane (knob 3) at 64 B
under the lane-pair loads (round 6; experiments build): interleaved rounds in one
process, HIP-event medians, every variant's output equal to the default's."""
import os as _os
_os.environ.setdefault("KVH_LIB", _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "libkvh_exp.so"))
import json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raikv_amd as kvh  # noqa: E402

torch.cuda.set_device(0)
L = int(sys.argv[1]) if len(sys.argv) > 1 else 64
n = 100_000_000
keys = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda")
out = torch.empty((n, 2), dtype=torch.int64, device="cuda")
ref = kvh.meow128_fixed(keys, L, kvh.STATIC_SEED).cpu()
# (tables, keys per lane); (0, 0) = the default
kpls = [(0, 0)] + [(nt, k) for nt in (4, 2) for k in (1, 2, 3, 4)]
same = {}
for k in kpls:
    kvh.lib.kvh_set_tuning(0, k[0]); kvh.lib.kvh_set_tuning(3, k[1])
    same[k] = bool(torch.equal(kvh.meow128_fixed(keys, L, kvh.STATIC_SEED).cpu(), ref))
del ref
res = {k: [] for k in kpls}
st = torch.cuda.current_stream()
for r in range(6):
    for k in kpls:
        kvh.lib.kvh_set_tuning(0, k[0]); kvh.lib.kvh_set_tuning(3, k[1])
        kvh.meow128_fixed(keys, L, kvh.STATIC_SEED, out=out)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
        for a, b in ev:
            a.record(st); kvh.meow128_fixed(keys, L, kvh.STATIC_SEED, out=out); b.record(st)
        torch.cuda.synchronize()
        res[k] += [a.elapsed_time(b) for a, b in ev]
kvh.lib.kvh_set_tuning(3, 0); kvh.lib.kvh_set_tuning(0, 0)
for k in kpls:
    t = float(np.median(res[k]))
    print(json.dumps({"L": L, "n": n, "tables": k[0] or "default", "keys_per_lane": k[1] or "default",
                      "median_ms": round(t, 4),
                      "Gkeys_s": round(n / t / 1e6, 2), "equals_default": same[k]}), flush=True)
