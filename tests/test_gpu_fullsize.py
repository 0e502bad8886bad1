"""GPU: the BASELINE.json configs at their full sizes, and key windows past
the 32-bit byte range.

Full-size batches cannot be hashed by the CPU oracle in seconds, so each one
is checked three ways (tests/ README of the tier: size-independent
properties): a seeded sample of >= 20,000 keys against the oracle
(oracle/meow_oracle.c, pinned to the reference's golden vectors); the whole
batch against an independent device kernel (the straight-line per-key
restatement k_seeded, or the generic runtime-length kernel); and
determinism.  Configs (BASELINE.json `configs`): C2 = 100M zipf 8-256 B keys
(4.87 GB of key bytes: offsets past 2^32), C3 = 50M x 32 B x 4 seeds,
C4 = 125M x 32 B (one GPU's shard of 1B) and the whole 1B x 32 B global
batch on one GPU.  C1 is in test_gpu_parity.py.

Window spans >= 4 GiB: the length-sorted kernels keep u32 window-relative
offsets; a window whose bytes span 4 GiB or more takes a u64 input-order
path (k_var6, k_crc_var_sorted).  Checked with 18 MiB keys (a 256-key window
holding 246 of them spans 4.3 GiB) against k_seeded / k_crc_var and the oracle.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle_lib import crc_sigs, load_oracle, orc_crc, orc_meow, orc_multiseed, orc_var  # noqa: E402

ORC = load_oracle()
crc_sigs(ORC)
STATIC = (0xA8E0BCC94D1855F5, 0xAD3BEC1E8DE4A1A3)
C3_SEEDS = [(1, 2), (3, 4), (5, 6), (7, 8)]


@pytest.fixture(scope="module")
def kvh():
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests must run on an MI355X")
    import raikv_amd
    return raikv_amd


def u64(t):
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint64)


def dev_u64(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).cuda()


def gather_keys(keys_dev, offs: np.ndarray, idx: np.ndarray):
    """Bytes of the keys idx (sorted) -> (flat host bytes, local offsets)."""
    a, e = offs[idx].astype(np.int64), offs[idx + 1].astype(np.int64)
    lens = e - a
    loc = np.zeros(len(idx) + 1, dtype=np.uint64)
    loc[1:] = np.cumsum(lens)
    pos = np.repeat(a - loc[:-1].astype(np.int64), lens) + np.arange(int(loc[-1]), dtype=np.int64)
    flat = keys_dev[torch.from_numpy(pos).cuda()].cpu().numpy()
    return flat, loc


def orc_sample(flat, loc, seed):
    return orc_var(ORC, np.ascontiguousarray(flat), loc, seed)


def test_c2_full_size_offsets_past_4gib(kvh):
    """C2 at full size: 100M zipf(0.99) 8-256 B keys, 4.87 GB of key bytes, so
    offsets and window starts run past 2^32.  Whole batch == k_seeded (u64
    literal restatement, per-key seeds); >= 20k keys (including every key of
    the windows around byte 2^32) == oracle; fixup; determinism."""
    from raikv_amd.workload import offsets_from_lengths, zipf_lengths
    n = 100_000_000
    offs = offsets_from_lengths(zipf_lengths(n, 8, 256, seed=3))
    nbytes = int(offs[-1])
    assert nbytes > (1 << 32) + (1 << 28)  # 4.72 GB
    g = torch.Generator(device="cuda")
    g.manual_seed(2024)
    keys = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda", generator=g)
    doff = dev_u64(offs)
    got = kvh.meow128_var(keys, doff, STATIC)
    again = kvh.meow128_var(keys, doff, STATIC)
    assert torch.equal(got, again)
    sd = torch.tensor(np.array(STATIC, dtype=np.uint64).view(np.int64), device="cuda").repeat(n, 1)
    lit = kvh.meow128_var_seeded(keys, doff, sd)
    assert torch.equal(got, lit), "k_var6 != k_seeded on the full C2 batch"
    del lit, again, sd
    h = u64(got)
    # sample: 20k random keys + the windows (256 keys) around byte 2^32 and the last ones
    rng = np.random.default_rng(17)
    w32 = int(np.searchsorted(offs, 1 << 32, side="right")) - 1  # key holding byte 2^32
    around = np.arange(max(0, (w32 // 256 - 1) * 256), min(n, (w32 // 256 + 2) * 256))
    idx = np.unique(np.concatenate([rng.choice(n, 20_000, replace=False), around, np.arange(n - 300, n)]))
    flat, loc = gather_keys(keys, offs, idx)
    np.testing.assert_array_equal(h[idx], orc_sample(flat, loc, STATIC))
    # KeyFragment fixup epilogue on the same batch
    fx = u64(kvh.meow128_var(keys, doff, STATIC, fixup=True))
    want = h.copy()
    want[:, 0] &= np.uint64(0x7FFFFFFFFFFFFFFF)
    want[want[:, 0] <= 1, 0] = 2
    np.testing.assert_array_equal(fx, want)


def test_c3_full_size_four_seeds(kvh):
    """C3 at full size: 50M x 32 B keys x 4 seeds (kv_hash_meow128_4_same_length_4_seed
    with one key in all slots).  Whole batch == four single-seed k_fixed
    launches; 20k keys == oracle."""
    n, L = 50_000_000, 32
    g = torch.Generator(device="cuda")
    g.manual_seed(33)
    keys = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    out = kvh.meow128_multiseed(keys, L, C3_SEEDS)
    assert out.shape == (n, 4, 2)
    for a, s in enumerate(C3_SEEDS):
        one = kvh.meow128_fixed(keys, L, s)
        assert torch.equal(out[:, a, :], one), f"seed slot {a}"
        del one
    idx = np.sort(np.random.default_rng(3).choice(n, 20_000, replace=False))
    kb = keys.view(n, L)[torch.from_numpy(idx).cuda()].cpu().numpy().reshape(-1)
    np.testing.assert_array_equal(u64(out)[idx], orc_multiseed(ORC, kb, L, C3_SEEDS))


def test_c4_full_shard(kvh):
    """C4: one GPU's shard of 1B 32-byte keys (125M).  Whole batch == the
    generic runtime-length kernel; 20k keys == oracle; the shard equals the
    same index range hashed inside a larger batch (sharding is layout-neutral)."""
    n, L = 125_000_000, 32
    g = torch.Generator(device="cuda")
    g.manual_seed(44)
    keys = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    out = kvh.meow128_fixed(keys, L, STATIC)
    prev = kvh.lib.kvh_set_tuning(2, 1)
    try:
        gen = kvh.meow128_fixed(keys, L, STATIC)
    finally:
        kvh.lib.kvh_set_tuning(2, prev)
    assert torch.equal(out, gen)
    del gen
    idx = np.sort(np.random.default_rng(4).choice(n, 20_000, replace=False))
    kb = keys.view(n, L)[torch.from_numpy(idx).cuda()].cpu().numpy().reshape(-1)
    h = u64(out)
    loc = np.arange(0, (len(idx) + 1) * L, L, dtype=np.uint64)
    np.testing.assert_array_equal(h[idx], orc_sample(kb, loc, STATIC))
    # rank 3 of 8 (index range 3n/8 .. 4n/8) hashed on its own == its slice
    from raikv_amd.workload import shard_range
    lo, hi = shard_range(n, 3, 8)
    part = kvh.meow128_fixed(keys[lo * L:hi * L], L, STATIC)
    assert torch.equal(part, out[lo:hi])


def test_c4g_one_global_batch_on_one_gpu(kvh):
    """C4 as BASELINE configs[4] states it (bench.py --config c4g, the N>1
    default): ONE global batch of 1B 32-byte keys (32 GB of keys, 16 GB of
    hashes), hashed by one launch on one MI355X.  20k sampled keys + the
    first/last keys == oracle; the whole batch == the generic runtime-length
    kernel; the index-range shards that bench.py gives ranks 0..7 of N = 2, 4
    and 8 hashed on their own == their slices of the one-launch result."""
    n, L = 1_000_000_000, 32
    g = torch.Generator(device="cuda")
    g.manual_seed(404)
    keys = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    out = kvh.meow128_fixed(keys, L, STATIC)
    prev = kvh.lib.kvh_set_tuning(2, 1)
    try:
        gen = kvh.meow128_fixed(keys, L, STATIC)
    finally:
        kvh.lib.kvh_set_tuning(2, prev)
    assert torch.equal(out, gen), "k_fixed != k_generic on the 1B batch"
    del gen
    rng = np.random.default_rng(404)
    idx = np.unique(np.concatenate([rng.choice(n, 20_000, replace=False), np.arange(0, 100), np.arange(n - 100, n)]))
    ti = torch.from_numpy(idx).cuda()
    kb = keys.view(n, L)[ti].cpu().numpy().reshape(-1)
    h = out[ti].cpu().numpy().view(np.uint64)
    loc = np.arange(0, (len(idx) + 1) * L, L, dtype=np.uint64)
    np.testing.assert_array_equal(h, orc_sample(kb, loc, STATIC))
    from raikv_amd.workload import shard_range
    for world in (2, 4, 8):
        for r in sorted({0, world // 2, world - 1}):
            lo, hi = shard_range(n, r, world)
            part = kvh.meow128_fixed(keys[lo * L:hi * L], L, STATIC)
            assert torch.equal(part, out[lo:hi]), (world, r)
            del part


def _big_window_batch():
    """300 keys of 18 MiB between small keys (10 zipf keys before, 1000
    after): the first 256-key window holds 246 of them and spans 4.3 GiB."""
    from raikv_amd.workload import zipf_lengths
    big = 18 << 20
    lens = np.concatenate([zipf_lengths(10, 8, 256, seed=5), np.full(300, big, np.uint32),
                           zipf_lengths(1000, 8, 256, seed=6)]).astype(np.uint64)
    offs = np.zeros(len(lens) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)
    n = len(lens)
    spans = [int(offs[min(i + 256, n)] - offs[i]) for i in range(0, n, 256)]
    assert max(spans) >= 1 << 32 and min(spans) < 1 << 32  # wide and ordinary windows
    return offs


def test_var_windows_spanning_4gib(kvh):
    offs = _big_window_batch()
    n = len(offs) - 1
    g = torch.Generator(device="cuda")
    g.manual_seed(55)
    keys = torch.randint(0, 256, (int(offs[-1]),), dtype=torch.uint8, device="cuda", generator=g)
    doff = dev_u64(offs)
    sd = torch.tensor(np.array(STATIC, dtype=np.uint64).view(np.int64), device="cuda").repeat(n, 1)
    lit = kvh.meow128_var_seeded(keys, doff, sd)
    for variant in (46, 0, 23):
        prev = kvh.lib.kvh_set_tuning(7, variant)
        try:
            got = kvh.meow128_var(keys, doff, STATIC)
        finally:
            kvh.lib.kvh_set_tuning(7, prev)
        assert torch.equal(got, lit), f"variant {variant}"
    h = u64(lit)
    # small keys + two 17 MiB keys against the oracle
    small = np.concatenate([np.arange(0, 10), np.arange(310, n)])
    flat, loc = gather_keys(keys, offs, small)
    np.testing.assert_array_equal(h[small], orc_sample(flat, loc, STATIC))
    for i in (10, 309):
        kb = keys[int(offs[i]):int(offs[i + 1])].cpu().numpy().tobytes()
        assert orc_meow(ORC, kb, *STATIC) == (int(h[i, 0]), int(h[i, 1])), i


def test_crc_windows_spanning_4gib(kvh):
    offs = _big_window_batch()
    n = len(offs) - 1
    g = torch.Generator(device="cuda")
    g.manual_seed(66)
    keys = torch.randint(0, 256, (int(offs[-1]),), dtype=torch.uint8, device="cuda", generator=g)
    doff = dev_u64(offs)
    res = {}
    for variant in (0, 6):
        prev = kvh.lib.kvh_set_tuning(14, variant)
        try:
            res[variant] = kvh.crc_c_var(keys, doff, 0x1234)
        finally:
            kvh.lib.kvh_set_tuning(14, prev)
    for v in (6,):
        assert torch.equal(res[v], res[0]), f"crc variant {v}"
    c = res[0].cpu().numpy().view(np.uint32)
    for i in list(range(0, 10, 3)) + [10, 250, 309] + list(range(310, n, 97)):
        kb = keys[int(offs[i]):int(offs[i + 1])].cpu().numpy().tobytes()
        assert orc_crc(ORC, kb, 0x1234) == int(c[i]), i
