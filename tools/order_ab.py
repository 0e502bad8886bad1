#!/usr/bin/env python3
"""A/B of the fixed-length chunk order (kvh_set_tuning(24, v), knob 24:
1 = static per-wave order, k_fixed; 2 = wave tickets, k_fixed_qw;
3/4/5 = k_fixed_q with 1/4/16 workgroup-rounds per ticket; 0 = the per-length
default) on the C1 / C4 / C64 shapes and the other multiples of 8, one process, interleaved
rounds after a 500 ms settle, outputs asserted equal.  One JSON line per
(shape, order).  c3 = C3 (32-byte keys, four seeds, k_fixed_lanes); f1 = the
fused hash + positions kernel (k_fixed_pos), f1p = positions from resident
hashes (k_positions), f4 = CRC32C of 16-byte keys (k_crc_fixed_ct), f4v = CRC32C
of the C2 zipf keys (k_crc_var_sorted); 20 / 33 / 50 B run k_fixed_rt."""
import json, os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raikv_amd as kvh  # noqa: E402

torch.cuda.set_device(0)
for kv in filter(None, os.environ.get("KNOBS", "").split(",")):  # e.g. KNOBS=3=2 (keys per lane)
    k, v = kv.split("=")
    assert kvh.lib.kvh_set_tuning(int(k), int(v)) >= 0, kv
shapes = [(16, 100_000_000), (32, 125_000_000), (64, 100_000_000), (8, 100_000_000), (24, 100_000_000),
          (40, 100_000_000), (48, 100_000_000), (56, 100_000_000), ("c3", 50_000_000), ("f1", 100_000_000),
          ("f1p", 100_000_000), ("f4", 100_000_000), (20, 100_000_000), (33, 100_000_000), (50, 100_000_000),
          ("f4v", 100_000_000), ("f3", 1 << 30)]
if len(sys.argv) > 1:  # a comma list of shape names; any other key length runs 100M keys of it
    known = {str(s[0]): s for s in shapes}
    shapes = [known[t] if t in known else (int(t), 100_000_000) for t in sys.argv[1].split(",")]
from raikv_amd.workload import C3_SEEDS  # noqa: E402
st = torch.cuda.current_stream()
VS = [int(x) for x in os.environ.get("ORDERS", "1,2").split(",")]
KN = 24  # the knob the A/B alternates; VARY=K:v1,v2 alternates knob K instead of the chunk order
if os.environ.get("VARY"):
    KN, vals = os.environ["VARY"].split(":")
    KN, VS = int(KN), [int(x) for x in vals.split(",")]
NAMES = {0: "default", 1: "static", 2: "wave_tickets", 3: "tickets_r1", 4: "tickets_r4", 5: "tickets_r16"}
g = torch.Generator(device="cuda")
g.manual_seed(7)
F1_GEOM = dict(map_size=64 << 30, hash_entry_size=64, hash_value_ratio=1.0, cuckoo_buckets=4, cuckoo_arity=4)
for L, n in shapes:
    tag = L if isinstance(L, str) else None
    L = 32 if tag == "c3" else 16 if tag else L
    keys = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    if tag == "c3":
        out = torch.empty((n, 4, 2), dtype=torch.int64, device="cuda")
        hash_ = lambda: kvh.meow128_multiseed(keys, L, list(C3_SEEDS), out=out)
    elif tag in ("f1", "f1p"):
        geom = kvh.HtGeom.from_map(**F1_GEOM)
        hashes = torch.empty((n, 2), dtype=torch.int64, device="cuda")
        out = torch.empty((n, geom.per_key), dtype=torch.int64, device="cuda")
        if tag == "f1":
            hash_ = lambda: kvh.meow128_fixed_positions(keys, L, kvh.STATIC_SEED, geom, hashes=hashes, out=out)
        else:
            kvh.meow128_fixed(keys, L, kvh.STATIC_SEED, out=hashes, fixup=True)
            hash_ = lambda: kvh.ht_positions(hashes, geom, out=out)
    elif tag == "f3":  # 1 GiB text -> tokens -> NUL-terminated span hashes (one kvh_tokenize_hash call)
        del keys
        r = torch.randint(0, 8, (n,), dtype=torch.uint8, device="cuda", generator=g)
        keys = torch.where(r == 0, 32, torch.where(r == 1, 10, 97 + r)).to(torch.uint8)
        del r
        out = None  # the call allocates; its hashes are what the A/B compares
        hash_ = lambda: kvh.tokenize_hash(keys, kvh.STATIC_SEED)[2]
    elif tag == "f4v":
        from raikv_amd.workload import zipf_lengths, offsets_from_lengths  # noqa: E402
        offs_np = offsets_from_lengths(zipf_lengths(n, 8, 256, seed=3))
        keys = torch.randint(0, 256, (int(offs_np[-1]),), dtype=torch.uint8, device="cuda", generator=g)
        offs = torch.from_numpy(offs_np.view(np.int64)).cuda()
        out = torch.empty((n,), dtype=torch.int32, device="cuda")
        hash_ = lambda: kvh.crc_c_var(keys, offs, 0, out=out)
    elif tag == "f4":
        out = torch.empty((n,), dtype=torch.int32, device="cuda")
        hash_ = lambda: kvh.crc_c_fixed(keys, L, 0, out=out)
    else:
        out = torch.empty((n, 2), dtype=torch.int64, device="cuda")
        hash_ = lambda: kvh.meow128_fixed(keys, L, kvh.STATIC_SEED, out=out)
    ref = None
    for v in VS:
        kvh.lib.kvh_set_tuning(KN, v)
        got = hash_()
        got = out if out is not None else got
        torch.cuda.synchronize()
        if ref is None:
            ref = got.clone()
        else:
            assert torch.equal(ref, got), f"order {v} differs at L={L}"
    del ref
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        hash_()
        torch.cuda.synchronize()
    res = {v: [] for v in VS}
    for r in range(int(os.environ.get("ROUNDS", "6"))):
        for v in VS:
            kvh.lib.kvh_set_tuning(KN, v)
            hash_()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
            for a, b in ev:
                a.record(st)
                hash_()
                b.record(st)
            torch.cuda.synchronize()
            res[v] += [a.elapsed_time(b) for a, b in ev]
    kvh.lib.kvh_set_tuning(KN, 0)
    for v in VS:
        ms = float(np.median(res[v]))
        print(json.dumps({"shape": tag or f"L{L}", "knobs": os.environ.get("KNOBS", ""), "key_len": L, "n": n, "order": NAMES[v] if KN == 24 else f"knob{KN}={v}", "median_ms": ms,
                          "min_ms": float(np.min(res[v])), "G_units_s": n / ms / 1e6}), flush=True)
    del keys, out
    hashes = None
    torch.cuda.empty_cache()
