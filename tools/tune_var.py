#!/usr/bin/env python3
"""A/B of the variable-length kernels (kvh_set_tuning(7, v)) on config C2."""
import os as _os  # research knobs live in the experiments build (make experiments)
_os.environ.setdefault("KVH_LIB", _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "libkvh_exp.so"))
import argparse, json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raikv_amd as kvh  # noqa: E402
from raikv_amd.workload import zipf_lengths, offsets_from_lengths  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=100_000_000)
ap.add_argument("--variants", default="0,5,6")
ap.add_argument("--rounds", type=int, default=3)
a = ap.parse_args()
torch.cuda.set_device(0)
offs = offsets_from_lengths(zipf_lengths(a.n, 8, 256, seed=3))
keys = torch.randint(0, 256, (int(offs[-1]),), dtype=torch.uint8, device="cuda")
doff = torch.from_numpy(offs.view(np.int64)).cuda()
out = torch.empty((a.n, 2), dtype=torch.int64, device="cuda")
vs = [int(v) for v in a.variants.split(",")]
res = {v: [] for v in vs}
ref = None
st = torch.cuda.current_stream()
for r in range(a.rounds):
    for v in vs:
        kvh.lib.kvh_set_tuning(7, v)
        kvh.meow128_var(keys, doff, kvh.STATIC_SEED, out=out)
        torch.cuda.synchronize()
        if ref is None: ref = out.clone()
        else: assert torch.equal(ref, out), v
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(3)]
        for e0, e1 in ev:
            e0.record(st); kvh.meow128_var(keys, doff, kvh.STATIC_SEED, out=out); e1.record(st)
        torch.cuda.synchronize()
        res[v] += [e0.elapsed_time(e1) for e0, e1 in ev]
byt = int(offs[-1]) + 8 * (a.n + 1) + 16 * a.n
for v in vs:
    t = float(np.median(res[v]))
    print(json.dumps({"var_kernel": v, "median_ms": t, "Gkeys_s": a.n / t / 1e6, "GBps_alg": byt / t / 1e6}))
