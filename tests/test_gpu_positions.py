"""GPU parity for SURVEY.md §8 row f1 (table positions): kvh_ht_positions
and the fused kvh_meow128_fixed_positions vs the reference's golden vectors
(tests/golden/cuckoo_*.npz, produced by ht_init.cpp + ht_cuckoo.cpp) and the
oracle (oracle/cuckoo_oracle.c).  Bit-exact.

Run on an MI355X:  python -m pytest tests -m gpu -x -q
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle_lib import cuckoo_fixtures, load_oracle, orc_fixed, orc_geom, orc_positions  # noqa: E402

ORC = load_oracle()
FIX = cuckoo_fixtures()
STATIC = (0xA8E0BCC94D1855F5, 0xAD3BEC1E8DE4A1A3)


@pytest.fixture(scope="module")
def kvh():
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests must run on an MI355X")
    import raikv_amd
    return raikv_amd


def dev_u64(a: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).cuda()


def host(t):
    torch.cuda.synchronize()
    a = t.cpu().numpy()
    return a.view(np.uint32) if a.dtype == np.int32 else a.view(np.uint64)


def geom_of(kvh, f):
    return kvh.HtGeom.from_map(f["map_size"], f["entry_size"], f["ratio"], f["buckets"], f["arity"])


@pytest.mark.parametrize("f", FIX, ids=[f["name"] for f in FIX])
def test_positions_golden(kvh, f):
    g = geom_of(kvh, f)
    h = dev_u64(f["hashes"])
    pos = kvh.ht_positions(h, g)
    np.testing.assert_array_equal(host(pos), f["pos"])
    p32 = kvh.ht_positions(h, g, pos32=True)
    np.testing.assert_array_equal(host(p32), f["pos"].astype(np.uint32))


@pytest.mark.parametrize("f", FIX, ids=[f["name"] for f in FIX])
def test_fused_golden(kvh, f):
    """keys16 -> hash -> fixup -> positions equals the reference's positions
    for the same keys' hashes (rows 1 .. 1+n of the fixture)."""
    g = geom_of(kvh, f)
    kb = f["keys16"]
    n = kb.size // 16
    want_h = f["hashes"][1:1 + n]
    want_p = f["pos"][1:1 + n]
    keys = torch.from_numpy(kb).cuda()
    for pos32 in (False, True):
        hh, pos = kvh.meow128_fixed_positions(keys, 16, f["seed"], g, pos32=pos32)
        np.testing.assert_array_equal(host(hh), want_h)
        np.testing.assert_array_equal(host(pos), want_p.astype(np.uint32) if pos32 else want_p)
    _, pos = kvh.meow128_fixed_positions(keys, 16, f["seed"], g, keep_hashes=False)
    np.testing.assert_array_equal(host(pos), want_p)


@pytest.mark.parametrize("L", [8, 16, 24, 32, 13, 64])
@pytest.mark.parametrize("arity,buckets", [(1, 1), (2, 4), (3, 2), (4, 4), (8, 2)])
def test_fused_all_shapes_vs_oracle(kvh, L, arity, buckets):
    # fused kernel (L 16/32, arity 1/2/4/8) and the two-pass path (the rest)
    rng = np.random.default_rng(L * 100 + arity)
    n = 5000
    kb = rng.integers(0, 256, n * L, dtype=np.uint8)
    g = kvh.HtGeom.from_map(8 << 20, 64, 1.0, buckets, arity)
    og = orc_geom(ORC, 8 << 20, 64, 1.0, buckets, arity)
    want_h = orc_fixed(ORC, kb, L, STATIC, fixup=True)
    want_p = orc_positions(ORC, og, want_h)
    hh, pos = kvh.meow128_fixed_positions(torch.from_numpy(kb).cuda(), L, STATIC, g)
    np.testing.assert_array_equal(host(hh), want_h)
    np.testing.assert_array_equal(host(pos), want_p)
    _, pos = kvh.meow128_fixed_positions(torch.from_numpy(kb).cuda(), L, STATIC, g, keep_hashes=False)
    np.testing.assert_array_equal(host(pos), want_p)


def test_unaligned_keys_take_two_pass_path(kvh):
    rng = np.random.default_rng(3)
    n = 3001
    buf = torch.from_numpy(rng.integers(0, 256, n * 16 + 8, dtype=np.uint8)).cuda()
    keys = buf[8:]  # 8-byte aligned only
    g = kvh.HtGeom.from_map(64 << 20, 64, 1.0, 4, 4)
    og = orc_geom(ORC, 64 << 20, 64, 1.0, 4, 4)
    kb = keys.cpu().numpy()
    want_h = orc_fixed(ORC, kb, 16, STATIC, fixup=True)
    hh, pos = kvh.meow128_fixed_positions(keys, 16, STATIC, g)
    np.testing.assert_array_equal(host(hh), want_h)
    np.testing.assert_array_equal(host(pos), orc_positions(ORC, og, want_h))


def test_edges_empty_single_ragged(kvh):
    g = kvh.HtGeom.from_map(64 << 20, 64, 1.0, 4, 4)
    og = orc_geom(ORC, 64 << 20, 64, 1.0, 4, 4)
    rng = np.random.default_rng(9)
    for n in (0, 1, 2, 63, 64, 65, 127, 129, 1000, 4097):
        h = rng.integers(0, 2 ** 64, size=(n, 2), dtype=np.uint64)
        pos = kvh.ht_positions(dev_u64(h) if n else torch.empty((0, 2), dtype=torch.int64, device="cuda"), g)
        assert tuple(pos.shape) == (n, 4)
        if n:
            np.testing.assert_array_equal(host(pos), orc_positions(ORC, og, h))


def test_huge_table_geometry(kvh):
    # a 2^35-entry table (2 TiB of 64 B entries): u64 ring arithmetic and
    # masks beyond 32 bits; geometry from the same restatement the fixtures pin
    rng = np.random.default_rng(21)
    h = rng.integers(0, 2 ** 64, size=(200_000, 2), dtype=np.uint64)
    for ms in (1 << 41, 3 << 40, 288 << 30, 255 << 30, 16 << 30):
        g = kvh.HtGeom.from_map(ms, 64, 1.0, 4, 4)
        og = orc_geom(ORC, ms, 64, 1.0, 4, 4)
        pos = kvh.ht_positions(dev_u64(h), g)
        np.testing.assert_array_equal(host(pos), orc_positions(ORC, og, h))


def test_full_size_fused_properties(kvh):
    """100M 16-byte keys, arity 4 (C1 batch feeding a 64 GiB cuckoo table):
    fused == hash kernel + positions kernel everywhere, slots in range and
    pairwise clash-free, plus an oracle spot check on a random sample."""
    n = 100_000_000
    gen = torch.Generator(device="cuda")
    gen.manual_seed(77)
    keys = torch.randint(0, 256, (n * 16,), dtype=torch.uint8, device="cuda", generator=gen)
    g = kvh.HtGeom.from_map(64 << 30, 64, 1.0, 4, 4)
    hh, pos = kvh.meow128_fixed_positions(keys, 16, STATIC, g)
    h2 = kvh.meow128_fixed(keys, 16, STATIC, fixup=True)
    assert torch.equal(hh, h2)
    pos2 = kvh.ht_positions(h2, g)
    assert torch.equal(pos, pos2)
    del h2, pos2
    hs = int(g.ht_size)
    assert int(pos.min()) >= 0 and int(pos.max()) < hs
    for i in range(4):
        for j in range(i):
            assert not bool(((pos[:, i] & 8191) == (pos[:, j] & 8191)).any())
            d = torch.remainder(pos[:, i] - pos[:, j], hs)
            assert bool(((d >= 4) & (hs - d >= 4)).all())
    idx = torch.randint(0, n, (20000,), device="cuda", generator=gen)
    kb = keys.view(n, 16)[idx].cpu().numpy().reshape(-1)
    og = orc_geom(ORC, 64 << 30, 64, 1.0, 4, 4)
    want_h = orc_fixed(ORC, kb, 16, STATIC, fixup=True)
    np.testing.assert_array_equal(host(hh[idx]), want_h)
    np.testing.assert_array_equal(host(pos[idx]), orc_positions(ORC, og, want_h))
