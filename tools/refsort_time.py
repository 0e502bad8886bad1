"""Timing of the exact-order sort (KVH_REF_ORDER, ht_refsort.hip) at ctest's
batch sizes, beside the reference's own kv_ht_radix_sort on one host core
(oracle/_ref ref_ht_sort_bench, the checker library; 64 GiB-map geometry as
bench.py's f2).  One JSON line per batch size: device ms per call (HIP events
around 50 calls on the current stream), the reference's ms per call, and the
default (total-order) engine's ms for comparison."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import raikv_amd as kvh  # noqa: E402
from oracle_lib import load_ref_ht  # noqa: E402  (checker / CPU baseline only)

ref = load_ref_ht()
geom = kvh.HtGeom.from_map(map_size=64 << 30, hash_entry_size=64, hash_value_ratio=1.0, cuckoo_buckets=4,
                           cuckoo_arity=4)
rng = np.random.default_rng(1)
for n in (1024, 4096, 16384, 65536):
    h = rng.integers(0, 2 ** 64, size=(n, 2), dtype=np.uint64)
    dh = torch.from_numpy(h.view(np.int64)).cuda()
    srt = kvh.HtSorter(geom, n)
    res = {"n": n}
    for name, ro in (("ref_order", True), ("total_order", False)):
        for _ in range(5):
            srt.sort(dh, dedup=True, ref_order=ro)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(50):
            srt.sort(dh, dedup=True, ref_order=ro)
        b.record()
        torch.cuda.synchronize()
        res[f"{name}_ms"] = a.elapsed_time(b) / 50
    if ref is not None:
        d = np.zeros(1, np.uint64)
        ts = [ref.ref_ht_sort_bench(geom.ht_size, geom.ht_mod_mask, geom.ht_mod_fraction, geom.ht_mod_shift,
                                    h.ctypes.data, n, d.ctypes.data) for _ in range(20)]
        res["reference_cpu_ms_1core"] = float(np.median(ts)) * 1e3
    print(json.dumps(res), flush=True)

# ctest's batch loop in one launch (kvh_ht_sort_batched): throughput over
# many 16K batches, one workgroup per batch, against the same sort on one core
for nb in (1, 64, 1024):
    n = nb * 16384
    h = rng.integers(0, 2 ** 64, size=(n, 2), dtype=np.uint64)
    dh = torch.from_numpy(h.view(np.int64)).cuda()
    for _ in range(3):
        kvh.ht_sort_batched(dh, geom, batch=16384, dedup=True)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    a.record()
    for _ in range(reps):
        kvh.ht_sort_batched(dh, geom, batch=16384, dedup=True)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    res = {"batched_16k": nb, "n": n, "ms": ms, "G_pairs_s": n / ms / 1e6}
    if ref is not None:
        d = np.zeros(1, np.uint64)
        hb = np.ascontiguousarray(h[:16384])
        t1 = float(np.median([ref.ref_ht_sort_bench(geom.ht_size, geom.ht_mod_mask, geom.ht_mod_fraction,
                                                    geom.ht_mod_shift, hb.ctypes.data, 16384, d.ctypes.data)
                              for _ in range(10)]))
        res["reference_cpu_G_pairs_s_1core"] = 16384 / t1 / 1e9
    print(json.dumps(res), flush=True)

# The batching front end of the drop-in (kvh_ht_radix_sort_batch, VERDICT r5
# item 8): nbatch host kv_ht_sort_t arrays of ctest's batch shape (~8K frags:
# its 64 KiB frag buffer fills first; and full 16K ones) in one call, wall
# clock per call including the pinned H2D / D2H copies and the host packing,
# against the reference's kv_ht_radix_sort on one host core per batch
import ctypes as C  # noqa: E402
import time  # noqa: E402


class SortT(C.Structure):  # kv_ht_sort_t (radix_sort.h:8-11)
    _fields_ = [("key", C.c_uint64), ("key2", C.c_uint64), ("item", C.c_void_p)]


for bsz in (8192, 16384):
    hb = rng.integers(0, 2 ** 64, size=(bsz, 2), dtype=np.uint64)
    d = np.zeros(1, np.uint64)
    t1 = float(np.median([ref.ref_ht_sort_bench(geom.ht_size, geom.ht_mod_mask, geom.ht_mod_fraction,
                                                geom.ht_mod_shift, hb.ctypes.data, bsz, d.ctypes.data)
                          for _ in range(20)])) if ref is not None else None
    for nb in (1, 8, 24, 64, 256):
        arrs = []
        for b in range(nb):
            ar = (SortT * bsz)()
            v = np.frombuffer(ar, dtype=np.uint64).reshape(-1, 3)
            v[:, :2] = rng.integers(0, 2 ** 64, size=(bsz, 2), dtype=np.uint64)
            v[:, 2] = np.arange(bsz, dtype=np.uint64)
            arrs.append(ar)
        ptrs = (C.c_void_p * nb)(*[C.addressof(a) for a in arrs])
        szs = (C.c_uint32 * nb)(*([bsz] * nb))
        for _ in range(3):
            assert kvh.lib.kvh_ht_radix_sort_batch(ptrs, szs, nb, C.byref(geom)) == 0
        ts = []
        for _ in range(10):
            t = time.perf_counter()
            assert kvh.lib.kvh_ht_radix_sort_batch(ptrs, szs, nb, C.byref(geom)) == 0
            ts.append(time.perf_counter() - t)
        ms = float(np.median(ts)) * 1e3
        res = {"radix_sort_batch": nb, "batch": bsz, "ms_per_call": ms, "ms_per_batch": ms / nb}
        if t1 is not None:
            res["reference_cpu_ms_per_batch_1core"] = t1 * 1e3
        print(json.dumps(res), flush=True)
