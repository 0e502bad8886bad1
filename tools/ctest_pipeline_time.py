#!/usr/bin/env python3
"""ctest's ingest on the device at bench.py's f3 size (1 GiB of text, ~201M
tokens): kvh_tokenize_hash, then ctest's batches (~8K frags each: its 64 KiB
frag buffer fills first) in kv_ht_radix_sort's exact order with duplicate
marking (kvh_ht_sort_segments).  Device time per stage (torch events,
medians of 5), beside the reference on one host core: ctest's tokenize +
frag + hash (oracle/_ref ref_ctest_ingest_bench via bench.py's leg) and
kv_ht_radix_sort + marking on 8K batches (ref_ht_sort_bench).
The batch cuts restart at every 256 KiB read block as ctest's do
(tests/ctest_batches.py); the tokens come from one pass over the whole text,
so a token running across a block end (at most one per 4096 blocks) is kept
whole here where ctest splits it.  The exact per-block form is
tests/test_gpu_ingest.py::test_ctest_pipeline_on_device."""
import json, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import raikv_amd as kvh  # noqa: E402
from ctest_batches import CTEST_BLOCK, ctest_block_batches  # noqa: E402
from oracle_lib import load_ref_ht  # noqa: E402  (CPU baseline only)

torch.cuda.set_device(0)
n = 1 << 30
g = torch.Generator(device="cuda"); g.manual_seed(1000)
r = torch.randint(0, 8, (n,), dtype=torch.uint8, device="cuda", generator=g)
text = torch.where(r == 0, 32, torch.where(r == 1, 10, 97 + r)).to(torch.uint8)
del r
geom = kvh.HtGeom.from_map(map_size=64 << 30, hash_entry_size=64, hash_value_ratio=1.0, cuckoo_buckets=4,
                           cuckoo_arity=4)
seed = kvh.STATIC_SEED
o, l, h = kvh.tokenize_hash(text, seed, 256)
ntok = l.numel()
ln, blk = l.cpu().numpy(), (o // CTEST_BLOCK).cpu().numpy()
edges = np.searchsorted(blk, np.arange(int(blk[-1]) + 2))
cuts = ctest_block_batches([ln[edges[b]:edges[b + 1]] for b in range(len(edges) - 1)])
dcuts = torch.from_numpy(cuts.view(np.int64)).cuda()
h = h.contiguous()
del o


def timed(f, reps=5):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); f(); b.record(); torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts))


kvh.ht_sort_segments(h, geom, dcuts, max_seg=16384, dedup=True)
t_th = timed(lambda: kvh.tokenize_hash(text, seed, 256, cap=ntok + 16))
t_sort = timed(lambda: kvh.ht_sort_segments(h, geom, dcuts, max_seg=16384, dedup=True))
_, _, dc = kvh.ht_sort_segments(h, geom, dcuts, max_seg=16384, dedup=True)
res = {"tokens": ntok, "batches": len(cuts) - 1, "mean_batch": ntok / (len(cuts) - 1),
       "dup_count": int(dc.sum().item()), "tokenize_hash_ms": t_th, "sort_segments_ms": t_sort,
       "device_tokens_per_s": ntok / (t_th + t_sort) * 1e3}
ref = load_ref_ht()
if ref is not None:
    hh = h[:8192].cpu().numpy().view(np.uint64).copy()
    d = np.zeros(1, np.uint64)
    t1 = float(np.median([ref.ref_ht_sort_bench(geom.ht_size, geom.ht_mod_mask, geom.ht_mod_fraction,
                                                geom.ht_mod_shift, hh.ctypes.data, 8192, d.ctypes.data)
                          for _ in range(20)]))
    res["reference_sort_tokens_per_s_1core"] = 8192 / t1
print(json.dumps(res), flush=True)
