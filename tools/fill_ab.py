#!/usr/bin/env python3
"""A/B of one library build against another (KVH_LIB selects it), one
process per library: HIP-event medians of the fixed-length hash (16 B: 4K,
1M and 100M keys; 64 B: 100M), CRC32C of 16-byte keys (100M) and the
variable-length hash (1M zipf keys).  Round 6: the table fill with its loads
batched (meow_dev.hpp fill_tables, crc32c.hip fill_crc) against the
word-at-a-time fill.  Usage: KVH_LIB=... python tools/fill_ab.py TAG"""
import json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raikv_amd as kvh  # noqa: E402
from raikv_amd.workload import zipf_lengths  # noqa: E402

torch.cuda.set_device(0)
tag = sys.argv[1]
st = torch.cuda.current_stream()


def timed(fn, reps=20):
    fn(); torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(st); fn(); b.record(st)
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


res = {"lib": tag}
k16 = torch.randint(0, 256, (100_000_000 * 16,), dtype=torch.uint8, device="cuda")
o16 = torch.empty((100_000_000, 2), dtype=torch.int64, device="cuda")
for n in (4096, 1_000_000, 100_000_000):
    res[f"fixed16_{n}"] = timed(lambda: kvh.meow128_fixed(k16[:n * 16], 16, kvh.STATIC_SEED, out=o16[:n]))
c32 = torch.empty(100_000_000, dtype=torch.int32, device="cuda")
res["crc16_100M"] = timed(lambda: kvh.crc_c_fixed(k16, 16, 7, out=c32))
res["crc16_4096"] = timed(lambda: kvh.crc_c_fixed(k16[:4096 * 16], 16, 7, out=c32[:4096]))
del k16
k64 = torch.randint(0, 256, (100_000_000 * 64,), dtype=torch.uint8, device="cuda")
res["fixed64_100M"] = timed(lambda: kvh.meow128_fixed(k64, 64, kvh.STATIC_SEED, out=o16))
del k64
lens = zipf_lengths(1_000_000)
offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
kv = torch.randint(0, 256, (int(offs[-1]) + 16,), dtype=torch.uint8, device="cuda")
do = torch.from_numpy(offs).cuda()
res["var_1M"] = timed(lambda: kvh.meow128_var(kv, do, kvh.STATIC_SEED))
print(json.dumps({k: (round(v, 5) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)
