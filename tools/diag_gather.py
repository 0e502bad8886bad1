#!/usr/bin/env python3
"""Diagnostic: is the length-sorted variable-length kernel bound by its
scattered key gathers?  Same zipf 8-256 B lengths twice: as generated, and
sorted ascending (a window's length order is then its address order, so a
wave's gathers coalesce).  Times kvh_crc_c_var and kvh_meow128_var on both."""
import json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raikv_amd as kvh  # noqa: E402
from raikv_amd.workload import zipf_lengths, offsets_from_lengths  # noqa: E402

torch.cuda.set_device(0)
n = 100_000_000
lens = zipf_lengths(n, 8, 256, seed=3)
st = torch.cuda.current_stream()
for name, ln in (("zipf", lens), ("zipf_sorted", np.sort(lens))):
    offs = offsets_from_lengths(ln)
    keys = torch.randint(0, 256, (int(offs[-1]),), dtype=torch.uint8, device="cuda")
    doff = torch.from_numpy(offs.view(np.int64)).cuda()
    co = torch.empty((n,), dtype=torch.int32, device="cuda")
    ho = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    for fn_name, fn in (("crc", lambda: kvh.crc_c_var(keys, doff, 0, out=co)),
                        ("meow", lambda: kvh.meow128_var(keys, doff, kvh.STATIC_SEED, out=ho))):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(7)]
        for a, b in ev:
            a.record(st); fn(); b.record(st)
        torch.cuda.synchronize()
        print(json.dumps({"data": name, "kernel": fn_name, "median_ms": float(np.median([a.elapsed_time(b) for a, b in ev]))}))
    del keys, doff, co, ho
