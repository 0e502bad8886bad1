#!/usr/bin/env python3
"""Per-phase wave cycles of k_var5 (stamped diagnostic build) on config C2."""
import os as _os  # research knobs live in the experiments build (make experiments)
_os.environ.setdefault("KVH_LIB", _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "libkvh_exp.so"))
import ctypes as C, json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raikv_amd as kvh  # noqa: E402
from raikv_amd.workload import zipf_lengths, offsets_from_lengths  # noqa: E402
torch.cuda.set_device(0)
n = 100_000_000
offs = offsets_from_lengths(zipf_lengths(n, 8, 256, seed=3))
keys = torch.randint(0, 256, (int(offs[-1]),), dtype=torch.uint8, device="cuda")
doff = torch.from_numpy(offs.view(np.int64)).cuda()
out = torch.empty((n, 2), dtype=torch.int64, device="cuda")
kvh.lib.kvh_set_tuning(7, 6)
kvh.lib.kvh_set_tuning(9, 1)
kvh.lib.kvh_debug_stamps.argtypes = [C.c_void_p, C.c_size_t]
for _ in range(3):
    kvh.meow128_var(keys, doff, kvh.STATIC_SEED, out=out)
torch.cuda.synchronize()
buf = np.zeros(4096 * 8, dtype=np.uint64)
assert kvh.lib.kvh_debug_stamps(buf.ctypes.data, buf.size) == 0
a = buf.reshape(4096, 8)[:, :6].astype(np.float64)
a = a[a.sum(1) > 0]
names = ["dma_issue", "count+scan+scatter", "wait_dma+barrier", "hash", "barrier_after_hash", "store+barrier"]
tot = a.sum(1).mean()
print(json.dumps({"waves": int(a.shape[0]), "mean_total_cycles": tot,
                  "phase_share": {nm: float(a[:, i].mean() / tot) for i, nm in enumerate(names)},
                  "hash_cycles_p10_p50_p90": [float(np.percentile(a[:, 3], q)) for q in (10, 50, 90)]}))
