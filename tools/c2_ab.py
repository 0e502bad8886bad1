#!/usr/bin/env python3
"""C2 A/B of variable-length kernels (kvh_set_tuning(7, v)), one process,
interleaved rounds after a 500 ms settle.  Variants whose outputs are hashes
are checked equal to the first variant; counter-only ablation builds (listed
in --ablations) are timed but not compared.  One JSON line per variant.

    KVH_LIB=tools/libkvh_exp.so python tools/c2_ab.py --variants 23,33,34 --ablations 28,29
"""
import os as _os  # research knobs live in the experiments build (make experiments)
_os.environ.setdefault("KVH_LIB", _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "libkvh_exp.so"))
import argparse, json, os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raikv_amd as kvh  # noqa: E402
from raikv_amd.workload import zipf_lengths, offsets_from_lengths  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=100_000_000)
ap.add_argument("--variants", default="23")
ap.add_argument("--ablations", default="")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--per", type=int, default=4, help="timed launches per variant per round")
ap.add_argument("--presorted", action="store_true",
                help="lengths already sorted by 16-byte class within each 256-key window (the sort ablation 61)")
a = ap.parse_args()
torch.cuda.set_device(0)
lens = zipf_lengths(a.n, 8, 256, seed=3)
if a.presorted:
    from c2_presort import presort_windows
    lens = presort_windows(lens)
offs = offsets_from_lengths(lens)
g = torch.Generator(device="cuda")
g.manual_seed(2024)
keys = torch.randint(0, 256, (int(offs[-1]),), dtype=torch.uint8, device="cuda", generator=g)
doff = torch.from_numpy(offs.view(np.int64)).cuda()
out = torch.empty((a.n, 2), dtype=torch.int64, device="cuda")
vs = [int(v) for v in a.variants.split(",") if v]
abl = [int(v) for v in a.ablations.split(",") if v]
allv = vs + abl
st = torch.cuda.current_stream()
ref = None
for v in allv:
    assert kvh.lib.kvh_set_tuning(7, v) >= 0, v
    out.zero_()
    kvh.meow128_var(keys, doff, kvh.STATIC_SEED, out=out)
    torch.cuda.synchronize()
    if v in abl:
        continue
    if ref is None:
        ref = out.clone()
    else:
        assert torch.equal(ref, out), f"variant {v} differs from {vs[0]}"
t_s = time.perf_counter()
while time.perf_counter() - t_s < 0.5:
    kvh.meow128_var(keys, doff, kvh.STATIC_SEED, out=out)
    torch.cuda.synchronize()
res = {v: [] for v in allv}
for r in range(a.rounds):
    for v in allv:
        kvh.lib.kvh_set_tuning(7, v)
        kvh.meow128_var(keys, doff, kvh.STATIC_SEED, out=out)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.per)]
        for e0, e1 in ev:
            e0.record(st); kvh.meow128_var(keys, doff, kvh.STATIC_SEED, out=out); e1.record(st)
        torch.cuda.synchronize()
        res[v] += [e0.elapsed_time(e1) for e0, e1 in ev]
kvh.lib.kvh_set_tuning(7, 23)
byt = int(offs[-1]) + 8 * (a.n + 1) + 16 * a.n
for v in allv:
    t = float(np.median(res[v]))
    print(json.dumps({"var_kernel": v, "hashes": v not in abl, "median_ms": round(t, 4),
                      "min_ms": round(float(np.min(res[v])), 4), "Gkeys_s": round(a.n / t / 1e6, 2),
                      "alg_TBps": round(byt / t / 1e9, 3)}), flush=True)
