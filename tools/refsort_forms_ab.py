#!/usr/bin/env python3
"""A/B of the exact-order batched forms beyond four batches per CU (experiments
build, knob 27: 0 = the four-wave form with 512-element wave nodes, 128 = the
two-wave form, 256 = the 256-thread form at four per CU) on
ctest's batches of bench.py's f3 text and on 4096 uniform 16K batches;
outputs asserted equal, medians of 5."""
import json, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import raikv_amd as kvh  # noqa: E402
from ctest_batches import ctest_batches  # noqa: E402

torch.cuda.set_device(0)
n = 1 << 30
g = torch.Generator(device="cuda"); g.manual_seed(1000)
r = torch.randint(0, 8, (n,), dtype=torch.uint8, device="cuda", generator=g)
text = torch.where(r == 0, 32, torch.where(r == 1, 10, 97 + r)).to(torch.uint8)
del r
geom = kvh.HtGeom.from_map(map_size=64 << 30, hash_entry_size=64, hash_value_ratio=1.0, cuckoo_buckets=4,
                           cuckoo_arity=4)
_, l, h = kvh.tokenize_hash(text, kvh.STATIC_SEED, 256)
del text
h = h.contiguous()
cuts = torch.from_numpy(ctest_batches(l.cpu().numpy()).view(np.int64)).cuda()
hu = h[:4096 * 16384].contiguous()


def timed(f, reps=5):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); f(); b.record(); torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts))


ref = {}
for v in (0, 128, 256, 0, 128, 256):
    assert kvh.lib.kvh_set_tuning(27, v) >= 0
    for name, f in (("ctest_segments", lambda: kvh.ht_sort_segments(h, geom, cuts, max_seg=16384, dedup=True)),
                    ("uniform_16k_x4096", lambda: kvh.ht_sort_batched(hu, geom, batch=16384, dedup=True))):
        out = f(); torch.cuda.synchronize()
        if name in ref:
            assert all(torch.equal(a, b) for a, b in zip(ref[name], out)), (name, v)
        else:
            ref[name] = out
        print(json.dumps({"knob27": v, "workload": name, "median_ms": timed(f)}), flush=True)
