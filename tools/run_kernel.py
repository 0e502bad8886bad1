#!/usr/bin/env python3
"""Run one workload's kernel a few times (profiling target for rocprofv3)."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raikv_amd as kvh  # noqa: E402
from raikv_amd.workload import C3_SEEDS, offsets_from_lengths, zipf_lengths  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c1")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--n", type=int, default=0)
ap.add_argument("--nt", type=int, default=0)
ap.add_argument("--kpl", type=int, default=0)
ap.add_argument("--var", type=int, default=-1)
ap.add_argument("--knob", action="append", default=[], help="kvh_set_tuning K=V (repeatable)")
ap.add_argument("--presorted", action="store_true", help="c2: lengths pre-sorted by class within each 256-key window")
a = ap.parse_args()
for kv in a.knob:
    k, v = kv.split("=")
    assert kvh.lib.kvh_set_tuning(int(k), int(v)) >= 0, kv
if a.nt:
    kvh.lib.kvh_set_tuning(0, a.nt)
if a.kpl:
    kvh.lib.kvh_set_tuning(3, a.kpl)
if a.var >= 0:
    kvh.lib.kvh_set_tuning(7, a.var)
torch.cuda.set_device(0)
g = torch.Generator(device="cuda")
g.manual_seed(1)
cfg = {"c1": (100_000_000, 16, 1), "c2": (100_000_000, 0, 1), "c3": (50_000_000, 32, 4), "c4": (125_000_000, 32, 1), "c64": (100_000_000, 64, 1), "c4g": (1_000_000_000, 32, 1),
       "f1": (100_000_000, 16, -1), "f1p": (100_000_000, 16, -2), "f4": (100_000_000, 16, -4),
       "f4v": (100_000_000, 0, -4), "f3": (1 << 30, 0, -3), "f2": (100_000_000, 16, -5)}
n, L, ar = cfg[a.config]
n = a.n or n
if ar == -5:  # table order, as bench.py's f2
    geom = kvh.HtGeom.from_map(64 << 30, 64, 1.0, 4, 4)
    keys = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    sh = kvh.meow128_fixed(keys, L, kvh.STATIC_SEED, fixup=True)
    del keys
    nd = n // 100
    sh[torch.randperm(n, device="cuda", generator=g)[:nd]] = sh[torch.randint(0, n, (nd,), device="cuda", generator=g)]
    si = torch.arange(n, dtype=torch.int64, device="cuda")
    sorter = kvh.HtSorter(geom, n)
    sho, sio = torch.empty_like(sh), torch.empty_like(si)
    f = lambda: sorter.sort(sh, si, dedup=True, out=sho, items_out=sio)
elif ar == -3:  # ingest: tokenize + NUL-terminated span hashes
    r = torch.randint(0, 8, (n,), dtype=torch.uint8, device="cuda", generator=g)
    text = torch.where(r == 0, 32, torch.where(r == 1, 10, 97 + r)).to(torch.uint8)
    del r

    f = lambda: kvh.tokenize_hash(text, kvh.STATIC_SEED, 256)  # as bench.py: one kvh_tokenize_hash call
elif ar == -4:  # CRC32C
    co = torch.empty((n,), dtype=torch.int32, device="cuda")
    if L == 0:
        offs = offsets_from_lengths(zipf_lengths(n, 8, 256, seed=3))
        keys = torch.randint(0, 256, (int(offs[-1]),), dtype=torch.uint8, device="cuda", generator=g)
        doff = torch.from_numpy(offs.view(np.int64)).cuda()
        f = lambda: kvh.crc_c_var(keys, doff, 0, out=co)
    else:
        keys = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
        f = lambda: kvh.crc_c_fixed(keys, L, 0, out=co)
elif ar < 0:  # table positions, geometry as bench.py F1_GEOM
    geom = kvh.HtGeom.from_map(64 << 30, 64, 1.0, 4, 4)
    keys = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    hh = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    pos = torch.empty((n, geom.per_key), dtype=torch.int64, device="cuda")
    if ar == -1:
        f = lambda: kvh.meow128_fixed_positions(keys, L, kvh.STATIC_SEED, geom, hashes=hh, out=pos)
    else:
        kvh.meow128_fixed(keys, L, kvh.STATIC_SEED, out=hh, fixup=True)
        f = lambda: kvh.ht_positions(hh, geom, out=pos)
elif L == 0:
    lens = zipf_lengths(n, 8, 256, seed=3)
    if a.presorted:
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from c2_presort import presort_windows
        lens = presort_windows(lens)
    offs = offsets_from_lengths(lens)
    keys = torch.randint(0, 256, (int(offs[-1]),), dtype=torch.uint8, device="cuda", generator=g)
    doff = torch.from_numpy(offs.view(np.int64)).cuda()
    f = lambda: kvh.meow128_var(keys, doff, kvh.STATIC_SEED)
else:
    keys = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    if ar == 1:
        f = lambda: kvh.meow128_fixed(keys, L, kvh.STATIC_SEED)
    else:
        f = lambda: kvh.meow128_multiseed(keys, L, list(C3_SEEDS[:ar]))
for _ in range(a.reps):
    f()
torch.cuda.synchronize()
print("ran", a.config, n, a.reps)
