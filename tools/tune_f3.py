#!/usr/bin/env python3
"""A/B of f3 ingest on bench.py's text (1 GiB, ~25 % separators, ~201M
tokens): kvh_tokenize + kvh_meow128_spans (two calls, the count known on the
host) against kvh_tokenize_hash (one call, the count read on the device).
Preallocated buffers; outputs asserted equal."""
import ctypes as C
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
ntok = kvh.tokenize(text, 256)[0].numel()
cap = ntok + 16
offs = torch.empty(cap, dtype=torch.int64, device="cuda")
lens = torch.empty(cap, dtype=torch.int32, device="cuda")
out = torch.empty((cap, 2), dtype=torch.int64, device="cuda")
cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
sb = kvh.lib.kvh_tokenize_scratch_bytes(n)
scr = torch.empty(sb // 8 + 1, dtype=torch.int64, device="cuda")
st = torch.cuda.current_stream()
s1, s2 = C.c_uint64(kvh.STATIC_SEED[0]), C.c_uint64(kvh.STATIC_SEED[1])
fl = kvh.KVH_FIXUP | kvh.KVH_NULTERM


def two():
    assert kvh.lib.kvh_tokenize(text.data_ptr(), n, 256, offs.data_ptr(), lens.data_ptr(), cap, cnt.data_ptr(),
                                scr.data_ptr(), sb, st.cuda_stream) == 0
    assert kvh.lib.kvh_meow128_spans(text.data_ptr(), offs.data_ptr(), lens.data_ptr(), ntok, s1, s2, out.data_ptr(),
                                     fl, st.cuda_stream) == 0


def fused():
    assert kvh.lib.kvh_tokenize_hash(text.data_ptr(), n, 256, s1, s2, fl, offs.data_ptr(), lens.data_ptr(),
                                     out.data_ptr(), cap, cnt.data_ptr(), scr.data_ptr(), sb, st.cuda_stream) == 0


ref, res = None, {"two_calls": [], "one_call": []}
for rnd in range(3):
    for name, f in (("two_calls", two), ("one_call", fused)):
        out.zero_(); f(); torch.cuda.synchronize()
        got = (offs[:ntok].clone(), lens[:ntok].clone(), out[:ntok].clone())
        if ref is None: ref = got
        else: assert all(torch.equal(a, b) for a, b in zip(ref, got)), name
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
        for a, b in ev:
            a.record(st); f(); b.record(st)
        torch.cuda.synchronize()
        res[name] += [a.elapsed_time(b) for a, b in ev]
for name, t in res.items():
    ms = float(np.median(t))
    print(json.dumps({"f3_path": name, "tokens": ntok, "median_ms": ms, "Gtok_s": ntok / ms / 1e6}))
