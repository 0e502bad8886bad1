#!/usr/bin/env python3
"""Throughput of the device frag-stream parse (kvh_frag_offsets: list
ranking) and of the one-call kvh_frags_hash on packed kv_key_frag_t streams
of f3-like tokens (1..14 bytes), at a few stream sizes."""
import json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raikv_amd as kvh  # noqa: E402

torch.cuda.set_device(0)
st = torch.cuda.current_stream()
for mib in (1, 16, 256):
    rng = np.random.default_rng(mib)
    target = mib << 20
    lens = rng.integers(1, 15, target // 6)
    recsz = 2 + lens + (lens & 1)
    cs = np.cumsum(recsz)
    k = int(np.searchsorted(cs, target))
    lens, recsz = lens[:k], recsz[:k]
    offs = np.concatenate([[0], np.cumsum(recsz)[:-1]]).astype(np.int64)
    buf = rng.integers(97, 123, int(recsz.sum()), dtype=np.uint8)
    for o, L in zip(offs[:0], lens[:0]):
        pass
    b16 = buf.view(np.uint8)
    b16[offs] = (lens & 255).astype(np.uint8)
    b16[offs + 1] = (lens >> 8).astype(np.uint8)
    d = torch.from_numpy(buf).cuda()
    got = kvh.frag_offsets(d)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy(), offs), mib
    res = {}
    for name, f in (("frag_offsets", lambda: kvh.frag_offsets(d, cap=k)),
                    ("frags_hash", lambda: kvh.frags_hash(d, kvh.STATIC_SEED, cap=k))):
        f(); torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
        for a, b in ev:
            a.record(st); f(); b.record(st)
        torch.cuda.synchronize()
        res[name] = float(np.median([a.elapsed_time(b) for a, b in ev]))
    print(json.dumps({"stream_MiB": mib, "records": k, **{n + "_ms": v for n, v in res.items()},
                      "Grec_s_parse": k / res["frag_offsets"] / 1e6, "Grec_s_hash": k / res["frags_hash"] / 1e6}))
