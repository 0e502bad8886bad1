#!/usr/bin/env python3
"""PCIe-inclusive host pipeline (kvh_meow128_fixed_host): chunk size sweep
(kvh_set_tuning knob 15, MiB of keys per chunk), pinned and pageable host
buffers; results checked against the device-resident kernel."""
import json, os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raikv_amd as kvh  # noqa: E402

torch.cuda.set_device(0)
n, L = 50_000_000, 16
hk = torch.randint(0, 256, (n * L,), dtype=torch.uint8).pin_memory()
ho = torch.empty((n, 2), dtype=torch.int64).pin_memory()
ref = kvh.meow128_fixed(hk.cuda(), L, kvh.STATIC_SEED).cpu()
import itertools
mibs = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "4,8,16,32,64").split(",")]
slots = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "8").split(",")]
for mib, sl in itertools.product(mibs, slots):
    kvh.lib.kvh_set_tuning(15, mib)
    kvh.lib.kvh_set_tuning(16, sl)
    kvh.meow128_fixed_host(hk.numpy(), L, kvh.STATIC_SEED, out=ho.numpy().view(np.uint64))
    assert torch.equal(ho, ref)
    ts = []
    for _ in range(4):
        t = time.perf_counter()
        kvh.meow128_fixed_host(hk.numpy(), L, kvh.STATIC_SEED, out=ho.numpy().view(np.uint64))
        ts.append(time.perf_counter() - t)
    dt = float(np.median(ts))
    print(json.dumps({"chunk_MiB": mib, "slots": sl, "pinned": True, "Ghash_s": n / dt / 1e9, "GBps_total": n * 32 / dt / 1e9}))
kvh.lib.kvh_set_tuning(15, 16)
pk = hk.numpy().copy()
po = np.empty((n, 2), dtype=np.uint64)
kvh.meow128_fixed_host(pk, L, kvh.STATIC_SEED, out=po)
t = time.perf_counter()
kvh.meow128_fixed_host(pk, L, kvh.STATIC_SEED, out=po)
dt = time.perf_counter() - t
assert np.array_equal(po, ref.numpy().view(np.uint64))
print(json.dumps({"chunk_MiB": 16, "pinned": False, "Ghash_s": n / dt / 1e9, "GBps_total": n * 32 / dt / 1e9}))
