#!/usr/bin/env python3
"""A/B of the tokenizers (kvh_set_tuning(19, v): 1 wave-chunked, 0
workgroup-chunked) on bench.py's f3 text (1 GiB, ~25 % separators); outputs
asserted equal.  Times kvh_tokenize (count, scan, emit) with torch events."""
import json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raikv_amd as kvh  # noqa: E402

torch.cuda.set_device(0)
n = 1 << 30
g = torch.Generator(device="cuda"); g.manual_seed(1000)
r = torch.randint(0, 8, (n,), dtype=torch.uint8, device="cuda", generator=g)
text = torch.where(r == 0, 32, torch.where(r == 1, 10, 97 + r)).to(torch.uint8)
del r
st = torch.cuda.current_stream()
cap = n // 4
d_offs = torch.empty(cap, dtype=torch.int64, device="cuda")
d_lens = torch.empty(cap, dtype=torch.int32, device="cuda")
cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
sb = kvh.lib.kvh_tokenize_scratch_bytes(n)
scr = torch.empty(sb // 8 + 1, dtype=torch.int64, device="cuda")


def tok():
    rc = kvh.lib.kvh_tokenize(text.data_ptr(), n, 256, d_offs.data_ptr(), d_lens.data_ptr(), cap, cnt.data_ptr(),
                              scr.data_ptr(), sb, st.cuda_stream)
    assert rc == 0, rc


ref, res = None, {0: [], 1: []}
for rnd in range(3):
    for v in (0, 1):
        kvh.lib.kvh_set_tuning(19, v)
        d_offs.zero_(); d_lens.zero_(); tok()
        torch.cuda.synchronize()
        k = int(cnt.item()); assert 0 < k < cap
        if ref is None: ref = (d_offs[:k].clone(), d_lens[:k].clone())
        else: assert torch.equal(ref[0], d_offs[:k]) and torch.equal(ref[1], d_lens[:k]), v
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
        for a, b in ev:
            a.record(st); tok(); b.record(st)
        torch.cuda.synchronize()
        res[v] += [a.elapsed_time(b) for a, b in ev]
kvh.lib.kvh_set_tuning(19, 1)
for v, t in res.items():
    ms = float(np.median(t))
    print(json.dumps({"tok_kernel": v, "tokens": ref[0].numel(), "median_ms": ms, "GB_s": n / ms / 1e6}))
