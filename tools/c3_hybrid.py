#!/usr/bin/env python3
"""C3 (50M x 32 B keys x 4 seeds): the product's k_fixed_lanes against the
research k_hybrid_lanes (tools/exp: a share of the keys through the
bitsliced VALU round, bs_meow.hpp) at several bitsliced shares, one process,
interleaved rounds after a 500 ms settle.  Outputs of every variant are
checked equal to the product's.  One JSON line per variant.

    python tools/c3_hybrid.py [--variants prod,0:4:2,125:4:2,250:4:2] [--profile permille:nbw:prio]
"""
import os as _os
_os.environ.setdefault("KVH_LIB", _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "libkvh_exp.so"))
import argparse, ctypes as C, json, os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raikv_amd as kvh  # noqa: E402
from raikv_amd.workload import C3_SEEDS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=50_000_000)
ap.add_argument("--variants", default="prod,0:4:2,125:2:2,125:4:2,250:4:2,250:4:0,500:8:2")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--profile", default="", help="run only this variant 5 times (rocprofv3 target)")
a = ap.parse_args()
torch.cuda.set_device(0)
L = 32
g = torch.Generator(device="cuda")
g.manual_seed(33)
keys = torch.randint(0, 256, (a.n * L,), dtype=torch.uint8, device="cuda", generator=g)
seeds = np.array(C3_SEEDS, dtype=np.uint64).reshape(-1)
out = torch.empty((a.n, 4, 2), dtype=torch.int64, device="cuda")
lib = kvh.lib
lib.kvh_exp_multiseed_hybrid.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                         C.c_uint32, C.c_void_p]
st = torch.cuda.current_stream()


def run(v):
    if v == "prod":
        kvh.meow128_multiseed(keys, L, list(C3_SEEDS), out=out)
        return
    pm, nbw, pr = (int(x) for x in v.split(":"))
    rc = lib.kvh_exp_multiseed_hybrid(keys.data_ptr(), a.n, seeds.ctypes.data, out.data_ptr(), pm, nbw, pr, 0,
                                      C.c_void_p(st.cuda_stream))
    assert rc == 0, (v, rc)


if a.profile:
    for _ in range(5):
        run(a.profile)
    torch.cuda.synchronize()
    sys.exit(0)
vs = a.variants.split(",")
run("prod")
torch.cuda.synchronize()
ref = out.clone()
for v in vs:
    out.zero_()
    run(v)
    torch.cuda.synchronize()
    assert torch.equal(out, ref), f"variant {v} differs from the product kernel"
del ref
t_s = time.perf_counter()
while time.perf_counter() - t_s < 0.5:
    run("prod")
    torch.cuda.synchronize()
res = {v: [] for v in vs}
for r in range(a.rounds):
    for v in vs:
        run(v)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(4)]
        for e0, e1 in ev:
            e0.record(st); run(v); e1.record(st)
        torch.cuda.synchronize()
        res[v] += [e0.elapsed_time(e1) for e0, e1 in ev]
for v in vs:
    t = float(np.median(res[v]))
    print(json.dumps({"variant": v, "bitsliced_permille": 0 if v == "prod" else int(v.split(":")[0]),
                      "median_ms": round(t, 4), "Ghash_s": round(4 * a.n / t / 1e6, 2),
                      "alg_TBps": round(a.n * 96 / t / 1e9, 3)}), flush=True)
