#!/usr/bin/env python3
"""Research build: k_var11 + k_var11_q (long-key deferral to queue kernels,
knob 7 = 40 / 41) and k_var12 (one kernel, knob 7 = 42 / 43) against k_var9 (knob 7 = 23)
on several length distributions (outputs pre-filled with a sentinel, so a
slot the queue kernel missed shows), then a C2 timing A/B."""
import argparse, json, os, sys
os.environ.setdefault("KVH_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "libkvh_exp.so"))  # research knobs
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raikv_amd as kvh  # noqa: E402
from raikv_amd.workload import zipf_lengths, offsets_from_lengths  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--variants", default="23,40,41")
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--n", type=int, default=100_000_000)
ap.add_argument("--skip-cases", action="store_true")
a = ap.parse_args()
torch.cuda.set_device(0)
vs = [int(v) for v in a.variants.split(",")]
rng = np.random.default_rng(5)


def run(keys, offs, v):
    kvh.lib.kvh_set_tuning(7, v)
    out = torch.full((offs.numel() - 1, 2), 0x5a5a5a5a5a5a5a5a, dtype=torch.int64, device="cuda")
    kvh.meow128_var(keys, offs, kvh.STATIC_SEED, out=out, fixup=True)
    torch.cuda.synchronize()
    return out


cases = {
    "zipf2M": zipf_lengths(2_000_000, 8, 256, seed=9),
    "all100": np.full(300_000, 100, np.int64),
    "cyc0_400": np.arange(500_000) % 401,
    "uni0_320": rng.integers(0, 321, 700_000),
    "long_heavy": np.where(rng.random(400_000) < 0.7, rng.integers(64, 320, 400_000), rng.integers(0, 64, 400_000)),
    "n5000": zipf_lengths(5000, 8, 256, seed=2),
    "n4096": zipf_lengths(4096, 0, 300, seed=4),
    "n100003": zipf_lengths(100_003, 0, 256, seed=6),
}
ok = True
for name, lens in ({} if a.skip_cases else cases).items():
    offs_np = offsets_from_lengths(np.asarray(lens, np.int64))
    keys = torch.randint(0, 256, (int(offs_np[-1]) + 1,), dtype=torch.uint8, device="cuda")[:int(offs_np[-1])]
    offs = torch.from_numpy(offs_np.view(np.int64)).cuda()
    ref = run(keys, offs, 23)
    for v in vs:
        got = run(keys, offs, v)
        eq = bool(torch.equal(ref, got))
        ok &= eq
        print(json.dumps({"case": name, "n": len(lens), "var": v, "equal": eq}), flush=True)
assert ok, "k_var11 differs"

offs_np = offsets_from_lengths(zipf_lengths(a.n, 8, 256, seed=3))
keys = torch.randint(0, 256, (int(offs_np[-1]),), dtype=torch.uint8, device="cuda")
offs = torch.from_numpy(offs_np.view(np.int64)).cuda()
ref = run(keys, offs, 23)
for v in vs:
    assert torch.equal(ref, run(keys, offs, v)), v
out = torch.empty((a.n, 2), dtype=torch.int64, device="cuda")
st = torch.cuda.current_stream()
res = {v: [] for v in vs}
t_s = __import__("time").perf_counter()
while __import__("time").perf_counter() - t_s < 0.5:
    kvh.meow128_var(keys, offs, kvh.STATIC_SEED, out=out); torch.cuda.synchronize()
for r in range(a.rounds):
    for v in vs:
        kvh.lib.kvh_set_tuning(7, v)
        kvh.meow128_var(keys, offs, kvh.STATIC_SEED, out=out)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
        for e0, e1 in ev:
            e0.record(st); kvh.meow128_var(keys, offs, kvh.STATIC_SEED, out=out); e1.record(st)
        torch.cuda.synchronize()
        res[v] += [e0.elapsed_time(e1) for e0, e1 in ev]
byt = int(offs_np[-1]) + 8 * (a.n + 1) + 16 * a.n
for v in vs:
    t = float(np.median(res[v]))
    print(json.dumps({"var_kernel": v, "median_ms": round(t, 4), "min_ms": round(float(np.min(res[v])), 4),
                      "Gkeys_s": round(a.n / t / 1e6, 2), "alg_TBps": round(byt / t / 1e9, 3)}), flush=True)
