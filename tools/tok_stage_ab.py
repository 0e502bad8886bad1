#!/usr/bin/env python3
"""A/B of the tokenizer emit pass's staging on bench.py's f3 text (1 GiB,
~25 % separators, no token near 2^30 bytes): max_token 256 runs the compact
int32 staging (k_tok2<true, true>), max_token 2^30 + 1 the u64 staging
(k_tok2<true, false>); on this text both keep the same tokens.  Outputs
poisoned and asserted equal; kvh_tokenize (count, scan, emit) and
kvh_tokenize_hash timed with torch events, interleaved, medians."""
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
st = torch.cuda.current_stream()
ntok = kvh.tokenize(text, 256)[0].numel()
cap = ntok + 16
d_offs = torch.empty(cap, dtype=torch.int64, device="cuda")
d_lens = torch.empty(cap, dtype=torch.int32, device="cuda")
out = torch.empty((cap, 2), dtype=torch.int64, device="cuda")
cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
sb = kvh.lib.kvh_tokenize_scratch_bytes(n)
scr = torch.empty(sb // 8 + 1, dtype=torch.int64, device="cuda")
s1, s2 = C.c_uint64(kvh.STATIC_SEED[0]), C.c_uint64(kvh.STATIC_SEED[1])
fl = kvh.KVH_FIXUP | kvh.KVH_NULTERM


def tok(mt):
    assert kvh.lib.kvh_tokenize(text.data_ptr(), n, mt, d_offs.data_ptr(), d_lens.data_ptr(), cap, cnt.data_ptr(),
                                scr.data_ptr(), sb, st.cuda_stream) == 0


def th(mt):
    assert kvh.lib.kvh_tokenize_hash(text.data_ptr(), n, mt, s1, s2, fl, d_offs.data_ptr(), d_lens.data_ptr(),
                                     out.data_ptr(), cap, cnt.data_ptr(), scr.data_ptr(), sb, st.cuda_stream) == 0


forms = {"c32": 256, "u64": (1 << 30) + 1}
ref, res = None, {(f, w): [] for f in forms for w in ("tokenize", "tokenize_hash")}
for rnd in range(4):
    for f, mt in forms.items():
        for w, fn in (("tokenize", tok), ("tokenize_hash", th)):
            for t_ in (d_offs, d_lens, out):
                t_.view(torch.uint8).fill_(0xA5)
            fn(mt); torch.cuda.synchronize()
            assert int(cnt.item()) == ntok
            if w == "tokenize_hash":
                got = (d_offs[:ntok].clone(), d_lens[:ntok].clone(), out[:ntok].clone())
                if ref is None: ref = got
                else: assert all(torch.equal(a, b) for a, b in zip(ref, got)), f
                del got
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(6)]
            for a, b in ev:
                a.record(st); fn(mt); b.record(st)
            torch.cuda.synchronize()
            res[(f, w)] += [a.elapsed_time(b) for a, b in ev]
for (f, w), t in res.items():
    print(json.dumps({"staging": f, "call": w, "median_ms": float(np.median(t)), "min_ms": float(np.min(t))}))
