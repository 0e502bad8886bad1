import sys, os, torch, numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raikv_amd as kvh
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
gen = torch.Generator(device="cuda"); gen.manual_seed(3)
keys = torch.randint(0, 256, (n * 16,), dtype=torch.uint8, device="cuda", generator=gen)
h = kvh.meow128_fixed(keys, 16, kvh.STATIC_SEED, fixup=True)
del keys
h0 = h.clone()
g = kvh.HtGeom.from_map(64 << 30, 64, 1.0, 4, 4)
print("scratch bytes", kvh.lib.kvh_ht_sort_scratch_bytes(n), flush=True)
srt = kvh.HtSorter(g, n)
print("scratch ptr", hex(srt.scratch.data_ptr()), "h ptr", hex(h.data_ptr()), flush=True)
oh, oi = srt.sort(h)
torch.cuda.synchronize()
print("h modified:", not torch.equal(h, h0), int((h != h0).any(1).sum()), flush=True)
print("oi perm:", torch.equal(torch.sort(oi).values, torch.arange(n, device="cuda")), flush=True)
bad = (oh != h0[oi]).any(1)
nb = int(bad.sum()); print("bad rows", nb, flush=True)
if nb:
    j = torch.nonzero(bad).flatten()[:10]
    print("j", j.tolist()); print("oi", oi[j].tolist()); print("oh", oh[j].tolist()); print("h0[oi]", h0[oi[j]].tolist())
    print("first bad", int(torch.nonzero(bad).flatten()[0]), "last bad", int(torch.nonzero(bad).flatten()[-1]))
# compare chunked gathers too
ok = all(torch.equal(oh[a:a + (1 << 23)], h0.index_select(0, oi[a:a + (1 << 23)])) for a in range(0, n, 1 << 23))
print("chunked index_select equal:", ok, flush=True)
