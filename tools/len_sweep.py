#!/usr/bin/env python3
"""Fixed-length throughput across the BASELINE metric's 16-64 B key range
(kvh_meow128_fixed, product library, device-resident).

    python tools/len_sweep.py [n] [lens] [variants]

n        keys per length (default 100M, the C1 batch size)
lens     comma list (default 16,24,32,48,64)
variants comma list of NT*10+U kernel shapes to A/B (e.g. 24,22,44,42;
         the round-3 sweeps also had a trailing p for a software-pipelined kernel,
         removed after it measured within 1 %), or
         "default" (the shipped choice only)

Per length: 500 ms settle (the post-idle power transient),
then per variant 5 warm-up + 20 timed launches with HIP events on the launch
stream; median and mean.  Outputs of every variant are checked against the
variable-length kernel on 4096 keys and against the default variant on the
whole batch.  One JSON line per (length, variant)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raikv_amd as kvh  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
lens = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [16, 24, 32, 48, 64]
variants = sys.argv[3].split(",") if len(sys.argv) > 3 else ["default"]
torch.cuda.set_device(0)
g = torch.Generator(device="cuda")
g.manual_seed(1)
maxL = max(lens)
keys = torch.randint(0, 256, (n * maxL,), dtype=torch.uint8, device="cuda", generator=g)
out = torch.empty((n, 2), dtype=torch.int64, device="cuda")
ref_out = torch.empty((n, 2), dtype=torch.int64, device="cuda")
st = torch.cuda.current_stream()
lib = kvh.lib


def setv(v):
    """'default', or NT*10+U"""
    if v == "default":
        lib.kvh_set_tuning(0, 0)
        lib.kvh_set_tuning(3, 0)
    else:
        v = int(v)
        assert lib.kvh_set_tuning(0, v // 10) >= 0 and lib.kvh_set_tuning(3, v % 10) >= 0


for L in sorted(lens):
    kb = keys[: n * L]
    setv("default")
    kvh.meow128_fixed(kb, L, kvh.STATIC_SEED, out=ref_out)
    m = 4096
    offs = torch.arange(0, (m + 1) * L, L, dtype=torch.int64, device="cuda")
    ref = kvh.meow128_var(kb[: m * L], offs, kvh.STATIC_SEED)
    assert torch.equal(ref, ref_out[:m]), L
    t_s = time.perf_counter()
    while time.perf_counter() - t_s < 0.5:
        kvh.meow128_fixed(kb, L, kvh.STATIC_SEED, out=out)
        torch.cuda.synchronize()
    for v in variants:
        try:
            setv(v)
            kvh.meow128_fixed(kb, L, kvh.STATIC_SEED, out=out)
        except Exception as e:  # a shape without an instance for this length
            print(json.dumps({"key_len": L, "variant": v, "error": repr(e)[:120]}), flush=True)
            continue
        torch.cuda.synchronize()
        assert torch.equal(out, ref_out), (L, v)
        for _ in range(5):
            kvh.meow128_fixed(kb, L, kvh.STATIC_SEED, out=out)
        ts = []
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
        for a, b in ev:
            a.record(st)
            kvh.meow128_fixed(kb, L, kvh.STATIC_SEED, out=out)
            b.record(st)
        torch.cuda.synchronize()
        ts = [a.elapsed_time(b) for a, b in ev]
        t = float(np.median(ts))
        alg = n * (L + 16)
        print(json.dumps({"key_len": L, "variant": v, "n": n, "ms_median": round(t, 4),
                          "ms_mean": round(float(np.mean(ts)), 4), "Ghash_s": round(n / t / 1e6, 1),
                          "alg_TBps": round(alg / t / 1e9, 3), "frac_spec": round(alg / t / 1e9 / 8.0, 3),
                          "frac_guide_copy": round(alg / t / 1e9 / 6.29, 3)}), flush=True)
setv("default")
