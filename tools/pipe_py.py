#!/usr/bin/env python3
"""Host pipeline rate from Python, with and without torch initialised first
(argv[1] = 'torch' to import and initialise torch before the library)."""
import sys, time, json, os
if len(sys.argv) > 2:
    os.sched_setaffinity(0, set(range(int(sys.argv[2]), int(sys.argv[2]) + 16)))
if len(sys.argv) > 1 and sys.argv[1] == "torch":
    import torch
    torch.cuda.init(); torch.zeros(1, device="cuda")
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raikv_amd as kvh  # noqa: E402
n, L = 50_000_000, 16
hk = kvh.host_empty((n * L,), np.uint8); hk[:] = 7
ho = kvh.host_empty((n, 2), np.uint64)
kvh.meow128_fixed_host(hk, L, (1, 2), out=ho)
ts = []
for _ in range(5):
    t = time.perf_counter(); kvh.meow128_fixed_host(hk, L, (1, 2), out=ho); ts.append(time.perf_counter() - t)
print(json.dumps({"args": sys.argv[1:], "cpu": os.sched_getaffinity(0).__len__(), "best_Ghash_s": n / min(ts) / 1e9, "median_Ghash_s": n / float(np.median(ts)) / 1e9}))
