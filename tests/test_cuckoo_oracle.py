"""CPU: the table-position oracle (oracle/cuckoo_oracle.c)
against the golden vectors the reference's own ht_init.cpp + ht_cuckoo.cpp
produced (tests/golden/cuckoo_*.npz), the product's host-side geometry
(kvh_ht_geom_init) against both, and the C-ABI's argument checks (no
device calls)."""
import ctypes as C

import numpy as np
import pytest

from oracle_lib import (OrcGeom, cuckoo_fixtures, load_oracle, load_ref_ht, orc_geom, orc_positions)

FIX = cuckoo_fixtures()


def test_fixture_set_complete():
    names = {f["name"] for f in FIX}
    assert {"kat64m_4x4", "srv64m_2p4", "tiny600_8x8", "lin64m_1", "big4g_4x4"} <= names
    assert len(FIX) >= 10


def test_hello_kat_positions():
    # RAIKV_STATIC_RANDOM seeds, 64 MiB map, arity 4, buckets 4
    f = [f for f in FIX if f["name"] == "kat64m_4x4"][0]
    assert int(f["geom"][3]) == 1041408
    assert [int(x) for x in f["pos"][0]] == [727478, 838349, 167394, 26629]
    lib = load_oracle()
    g = orc_geom(lib, 64 << 20, 64, 1.0, 4, 4)
    h1 = 0x2aa73a1eeb0b2d45 & ((1 << 63) - 1)  # README KAT hash, fixed up
    pos = orc_positions(lib, g, np.array([[h1, 0xfd102121185ce157]], dtype=np.uint64))
    assert [int(x) for x in pos[0]] == [727478, 838349, 167394, 26629]


@pytest.mark.parametrize("f", FIX, ids=[f["name"] for f in FIX])
def test_oracle_matches_reference_fixture(f):
    lib = load_oracle()
    g = orc_geom(lib, f["map_size"], f["entry_size"], f["ratio"], f["buckets"], f["arity"])
    assert (g.ht_mod_mask, g.ht_mod_fraction, g.ht_mod_shift, g.ht_size) == tuple(int(x) for x in f["geom"])
    pos = orc_positions(lib, g, f["hashes"])
    assert pos.shape == f["pos"].shape
    np.testing.assert_array_equal(pos, f["pos"])


@pytest.mark.parametrize("f", FIX, ids=[f["name"] for f in FIX])
def test_product_geometry_matches_reference(f):
    import raikv_amd as kvh
    g = kvh.HtGeom.from_map(f["map_size"], f["entry_size"], f["ratio"], f["buckets"], f["arity"])
    assert (g.ht_mod_mask, g.ht_mod_fraction, g.ht_mod_shift, g.ht_size) == tuple(int(x) for x in f["geom"])
    assert g.per_key == f["pos"].shape[1]
    # host ht_mod mirror == reference start slot
    for h, p in zip(f["hashes"][:50], f["pos"][:50]):
        assert g.ht_mod(int(h[0])) == int(p[0])


def test_product_geometry_matches_oracle_over_sizes():
    import raikv_amd as kvh
    lib = load_oracle()
    rng = np.random.default_rng(5)
    sizes = [int(x) for x in rng.integers(1 << 20, 1 << 40, 300)] + [(1 << k) + 12345 for k in range(20, 49)]
    for ms in sizes:
        for es, ratio in ((64, 1.0), (128, 0.5), (64, 0.37)):
            g = kvh.HtGeom.from_map(ms, es, ratio, 4, 4)
            o = orc_geom(lib, ms, es, ratio, 4, 4)
            assert (g.ht_size, g.ht_mod_mask, g.ht_mod_fraction, g.ht_mod_shift) == \
                (o.ht_size, o.ht_mod_mask, o.ht_mod_fraction, o.ht_mod_shift), (ms, es, ratio)
            top = (g.ht_mod_mask * g.ht_mod_fraction) >> g.ht_mod_shift
            assert g.ht_size // 2 < top < g.ht_size


def test_oracle_vs_reference_random_geometries():
    ref = load_ref_ht()
    if ref is None:
        pytest.skip("oracle/_ref/libkvref_ht.so not built (reference tree absent)")
    lib = load_oracle()
    rng = np.random.default_rng(11)
    hashes = rng.integers(0, 2 ** 64, size=(2000, 2), dtype=np.uint64)
    for _ in range(12):
        ms = int(rng.integers(600 << 10, 48 << 20))
        b = int(rng.integers(2, 9))
        a = int(rng.integers(2, 9))
        g = orc_geom(lib, ms, 64, 1.0, b, a)
        if g.ht_size < 4 * a * (2 * b):
            continue
        pos = np.zeros(len(hashes) * a, dtype=np.uint64)
        geom = np.zeros(4, dtype=np.uint64)
        assert ref.ref_cuckoo_positions(ms, 64, 1.0, b, a, hashes.ctypes.data, len(hashes), pos.ctypes.data,
                                        geom.ctypes.data) == 0
        np.testing.assert_array_equal(orc_positions(lib, g, hashes), pos.reshape(-1, a))


def test_positions_are_clash_free():
    # every pair of a key's slots differs in the 13-bit index and is at
    # least cuckoo_buckets apart on the ring (ht_cuckoo.cpp:56-76)
    for f in FIX:
        if f["pos"].shape[1] < 2:
            continue
        p = f["pos"].astype(np.int64)
        hs, b = int(f["geom"][3]), f["buckets"]
        for i in range(p.shape[1]):
            for j in range(i):
                assert not np.any((p[:, i] & 8191) == (p[:, j] & 8191)), f["name"]
                d = (p[:, i] - p[:, j]) % hs
                assert np.all((d >= b) & (hs - d >= b)), f["name"]
        assert np.all(p < hs)


def test_capi_rejects_bad_geometry_without_device():
    import raikv_amd as kvh
    lib = kvh.lib
    g = kvh.HtGeom.from_map(64 << 20, 64, 1.0, 4, 4)
    bad = kvh.HtGeom(); C.memmove(C.byref(bad), C.byref(g), C.sizeof(g))
    bad.ht_mod_fraction = bad.ht_mod_fraction * 4  # ht_mod would leave ht[]
    assert lib.kvh_ht_positions(None, 10, C.byref(bad), None, 0, None) == -22
    assert lib.kvh_ht_positions(None, 10, None, None, 0, None) == -22
    tiny = kvh.HtGeom.from_map((448 << 10) + 64 * 40, 64, 1.0, 8, 8)  # no room for 8 clash-free slots
    assert lib.kvh_ht_positions(None, 10, C.byref(tiny), None, 0, None) == -22
    big = kvh.HtGeom.from_map(1 << 40, 64, 1.0, 4, 4)  # > 2^32 slots: no u32 output
    assert lib.kvh_ht_positions(None, 10, C.byref(big), None, kvh.KVH_POS32, None) == -22
    assert lib.kvh_ht_positions(None, 0, C.byref(g), None, 0, None) == 0  # n == 0 is a no-op
    assert lib.kvh_ht_positions(None, 10, C.byref(g), None, 0, None) == -22  # NULL buffers
    assert lib.kvh_ht_geom_init(1000, 64, 1.0, 4, 4, C.byref(kvh.HtGeom())) == -22  # map smaller than header
    assert lib.kvh_positions_per_key(None) == 0
    assert kvh.HtGeom.from_map(64 << 20, 64, 1.0, 1, 4).per_key == 1  # buckets <= 1: linear probe
    assert kvh.HtGeom.from_map(64 << 20, 64, 1.0, 4, 1).per_key == 1
