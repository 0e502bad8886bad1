#!/usr/bin/env python3
"""f4v A/B (round 6): the length-sorted kernel that gathers keys from global
memory (knob 14 = 6) against windows staged in LDS (knob 14 = 7), on the f4v
shape (100M zipf 8-256 B keys) and on other length mixes; outputs asserted
equal; interleaved rounds in one process, HIP-event medians."""
import os as _os  # knob 14 = 7 lives in the experiments build (make experiments)
_os.environ.setdefault("KVH_LIB", _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "libkvh_exp.so"))
import json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raikv_amd as kvh  # noqa: E402
from raikv_amd.workload import zipf_lengths, offsets_from_lengths  # noqa: E402

torch.cuda.set_device(0)
st = torch.cuda.current_stream()
rng = np.random.default_rng(9)
cases = {
    "f4v_zipf_8_256_100M": zipf_lengths(100_000_000, 8, 256, seed=3),
    "uniform_0_300_4M": rng.integers(0, 301, 4_000_000).astype(np.uint64),
    "fixed_8_50M": np.full(50_000_000, 8, np.uint64),
    "long_1k_4k_200K": rng.integers(1024, 4097, 200_000).astype(np.uint64),
    "mixed_big_1M": np.where(rng.random(1_000_000) < 0.01, 20000, rng.integers(0, 64, 1_000_000)).astype(np.uint64),
}
for name, lens in cases.items():
    offs = offsets_from_lengths(lens)
    g = torch.Generator(device="cuda").manual_seed(7)
    keys = torch.randint(0, 256, (int(offs[-1]) + 1,), dtype=torch.uint8, device="cuda", generator=g)
    doff = torch.from_numpy(offs.view(np.int64)).cuda()
    n = len(lens)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    res, ref = {}, None
    for v in (6, 7):
        kvh.lib.kvh_set_tuning(14, v)
        o = kvh.crc_c_var(keys, doff, 0x1234).cpu()
        if ref is None:
            ref = o
        res[v] = {"equal": bool(torch.equal(o, ref)), "t": []}
    for r in range(5):
        for v in (6, 7):
            kvh.lib.kvh_set_tuning(14, v)
            kvh.crc_c_var(keys, doff, 0x1234, out=out)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(4)]
            for a, b in ev:
                a.record(st); kvh.crc_c_var(keys, doff, 0x1234, out=out); b.record(st)
            torch.cuda.synchronize()
            res[v]["t"] += [a.elapsed_time(b) for a, b in ev]
    kvh.lib.kvh_set_tuning(14, 6)
    row = {"case": name, "n": n, "bytes": int(offs[-1])}
    for v in (6, 7):
        t = float(np.median(res[v]["t"]))
        row[f"k{v}_ms"] = round(t, 4)
        row[f"k{v}_equal"] = res[v]["equal"]
    row["speedup"] = round(row["k6_ms"] / row["k7_ms"], 3)
    print(json.dumps(row), flush=True)
    del keys, doff, out
    torch.cuda.empty_cache()
